// String-column kernels for gfx950: predicates against literals, byte gathers (compaction / concat),
// CONCAT of views and literals, integer formatting, case mapping and the DataX `stringToTimestamp` UDF
// (reference: DataProcessing/datax-utility/src/main/scala/datax/utility/ConcurrentDateFormat.scala:14-62).
//
// Strings are views (start, len) into a byte arena; producing kernels are two-pass (length, then exclusive scan
// on the stream, then write), so no kernel ever needs dynamic allocation.
#include "dxa_common.h"
#include "decimal_dd.h"
#include "dxa_ts.h"
#include <stdlib.h>

namespace {

// op: 0 ==, 1 !=, 2 <, 3 <=, 4 >, 5 >= (byte-wise lexicographic, i.e. UTF-8 code-point order), 6 startsWith,
//     7 endsWith, 8 contains
__global__ void str_cmp_lit_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                   const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ lit,
                                   int32_t lit_len, int32_t op, uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    bool r = false;
    if (op <= 5) {
      if (op <= 1 && l != lit_len) {
        r = (op == 1);
      } else {
        const int32_t m = l < lit_len ? l : lit_len;
        int c = 0;
        for (int32_t k = 0; k < m; ++k) {
          if (s[k] != lit[k]) { c = (int)s[k] - (int)lit[k]; break; }
        }
        if (c == 0) c = (l > lit_len) - (l < lit_len);
        switch (op) {
          case 0: r = c == 0; break;
          case 1: r = c != 0; break;
          case 2: r = c < 0; break;
          case 3: r = c <= 0; break;
          case 4: r = c > 0; break;
          default: r = c >= 0; break;
        }
      }
    } else if (op == 6 || op == 7) {
      if (l >= lit_len) {
        const uint8_t* b = op == 6 ? s : s + (l - lit_len);
        r = true;
        for (int32_t k = 0; k < lit_len; ++k)
          if (b[k] != lit[k]) { r = false; break; }
      }
    } else {
      for (int32_t st = 0; st + lit_len <= l && !r; ++st) {
        bool m = true;
        for (int32_t k = 0; k < lit_len; ++k)
          if (s[st + k] != lit[k]) { m = false; break; }
        r = m;
      }
    }
    out[i] = r ? 1 : 0;
  }
}

// Column-vs-column ordering comparison (op: 2 <, 3 <=, 4 >, 5 >=), byte-wise (UTF-8 code point) order: 8 bytes at
// a time as big-endian words, then length.
__device__ __forceinline__ uint64_t be_chunk(const uint8_t* s, int32_t len, int32_t off) {
  uint64_t v = 0;
  const int32_t m = len - off < 8 ? len - off : 8;
  for (int32_t b = 0; b < m; ++b) v |= (uint64_t)s[off + b] << (56 - 8 * b);
  return v;
}

__global__ void str_cmp_col_kernel(const uint8_t* __restrict__ aa, const int64_t* __restrict__ as,
                                   const int32_t* __restrict__ al, const uint8_t* __restrict__ ba,
                                   const int64_t* __restrict__ bs, const int32_t* __restrict__ bl, int64_t n,
                                   int32_t op, uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* x = aa + as[i];
    const uint8_t* y = ba + bs[i];
    const int32_t lx = al[i], ly = bl[i];
    const int32_t m = lx < ly ? lx : ly;
    int c = 0;
    for (int32_t off = 0; off < m && c == 0; off += 8) {
      const uint64_t u = be_chunk(x, m, off), v = be_chunk(y, m, off);
      c = (u > v) - (u < v);
    }
    if (c == 0) c = (lx > ly) - (lx < ly);
    bool r;
    switch (op) {
      case 2: r = c < 0; break;
      case 3: r = c <= 0; break;
      case 4: r = c > 0; break;
      default: r = c >= 0; break;
    }
    out[i] = r ? 1 : 0;
  }
}

// Column-vs-column equality (join residuals, string = string predicates).
__global__ void str_eq_col_kernel(const uint8_t* __restrict__ aa, const int64_t* __restrict__ as,
                                  const int32_t* __restrict__ al, const uint8_t* __restrict__ ba,
                                  const int64_t* __restrict__ bs, const int32_t* __restrict__ bl, int64_t n,
                                  uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = al[i];
    bool r = l == bl[i];
    if (r) {
      const uint8_t* a = aa + as[i];
      const uint8_t* b = ba + bs[i];
      for (int32_t k = 0; k < l; ++k)
        if (a[k] != b[k]) { r = false; break; }
    }
    out[i] = r;
  }
}

// Copy each view's bytes to dst + dst_off[i] (compaction / concat of arenas), one lane per string: window panes and exchanges compact millions of short strings (device
// types, regions, ids: 4-20 B), where a wave per string leaves 60 of 64 lanes idle.  Each lane copies its string
// with unaligned 8-byte global loads/stores and a 4/2/1-byte tail (stores never touch a neighbour's bytes);
// strings longer than 128 B are copied afterwards by the whole wave, one at a time (ballot loop).
// Window flow: 19 gathers of 1 M strings per batch took 730 us with the wave-per-string kernel.
typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint16_t u16u __attribute__((aligned(1)));
#define SG1 __attribute__((address_space(1)))

__device__ __forceinline__ void copy_short(const SG1 uint8_t* s, SG1 uint8_t* d, int32_t l) {
  int32_t k = 0;
  for (; k + 8 <= l; k += 8) *(SG1 u64u*)(d + k) = *(const SG1 u64u*)(s + k);
  if (k + 4 <= l) { *(SG1 u32u*)(d + k) = *(const SG1 u32u*)(s + k); k += 4; }
  if (k + 2 <= l) { *(SG1 u16u*)(d + k) = *(const SG1 u16u*)(s + k); k += 2; }
  if (k < l) d[k] = s[k];
}

__global__ __launch_bounds__(256) void str_gather_lane_kernel(const uint8_t* __restrict__ arena,
                                                              const int64_t* __restrict__ starts,
                                                              const int32_t* __restrict__ lens, int64_t n,
                                                              const int64_t* __restrict__ dst_off,
                                                              uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const SG1 uint8_t* s = nullptr;
  SG1 uint8_t* d = nullptr;
  int32_t l = 0;
  if (i < n) {
    l = lens[i];
    s = (const SG1 uint8_t*)arena + starts[i];
    d = (SG1 uint8_t*)dst + dst_off[i];
  }
  const bool lng = l > 128;
  if (!lng && l > 0) copy_short(s, d, l);
  uint64_t m = __ballot(lng);
  const int lane = threadIdx.x & 63;
  while (m) {
    const int j = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const SG1 uint8_t* sj = (const SG1 uint8_t*)__shfl((uint64_t)(uintptr_t)s, j);
    SG1 uint8_t* dj = (SG1 uint8_t*)__shfl((uint64_t)(uintptr_t)d, j);
    const int32_t lj = __shfl(l, j);
    for (int32_t k = lane; k < lj; k += 64) dj[k] = sj[k];
  }
}

// Many string gathers in one launch: part p copies its rows [row0_p, row0_{p+1}) of the launch's row space from
// its own arena into its own destination (dst + dst_off[r]).  Used for row-concatenation (parts share one dst and
// consecutive offset ranges) and for compacting several columns at once (each its own dst) — one launch instead of
// one per part.  Descriptors travel in the kernel argument block; a lane finds its part by a short scan of row0.
constexpr int kMaxStrParts = 32;

struct StrPart {
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
  const int64_t* dst_off;
  uint8_t* dst;
  int64_t row0;
  // compaction form (dst_off null): the destination offset is incl[r] - lens[r] of an inclusive byte scan, and is
  // also stored to ex_out[r] (the compacted column's starts) — no separate subtraction pass
  const int64_t* incl;
  int64_t* ex_out;
};

struct StrParts {
  StrPart p[kMaxStrParts];
  int32_t k;
  int64_t total;
};

__global__ __launch_bounds__(256) void str_gather_parts_kernel(const StrParts a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const SG1 uint8_t* s = nullptr;
  SG1 uint8_t* d = nullptr;
  int32_t l = 0;
  if (i < a.total) {
    int q = 0;
    for (int t = 1; t < a.k; ++t) q = i >= a.p[t].row0 ? t : q;
    const StrPart& P = a.p[q];
    const int64_t r = i - P.row0;
    l = P.lens[r];
    s = (const SG1 uint8_t*)P.arena + P.starts[r];
    int64_t doff;
    if (P.dst_off) {
      doff = P.dst_off[r];
    } else {
      doff = P.incl[r] - (int64_t)l;
      P.ex_out[r] = doff;
    }
    d = (SG1 uint8_t*)P.dst + doff;
  }
  const bool lng = l > 128;
  if (!lng && l > 0) copy_short(s, d, l);
  uint64_t m = __ballot(lng);
  const int lane = threadIdx.x & 63;
  while (m) {
    const int j = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const SG1 uint8_t* sj = (const SG1 uint8_t*)__shfl((uint64_t)(uintptr_t)s, j);
    SG1 uint8_t* dj = (SG1 uint8_t*)__shfl((uint64_t)(uintptr_t)d, j);
    const int32_t lj = __shfl(l, j);
    for (int32_t k = lane; k < lj; k += 64) dj[k] = sj[k];
  }
}

// CONCAT(part_0, …, part_{k-1}); each part is either a column view or a literal.  Null in any column part → null.
struct ConcatPart {
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
  const uint8_t* valid;
  const uint8_t* lit;
  int32_t lit_len;
  int32_t is_lit;
};

__global__ void concat_len_kernel(const ConcatPart* __restrict__ parts, int32_t k, int64_t n,
                                  int64_t* __restrict__ out_len, uint8_t* __restrict__ out_valid) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t l = 0;
    bool ok = true;
    for (int32_t p = 0; p < k; ++p) {
      const ConcatPart& c = parts[p];
      if (c.is_lit) { l += c.lit_len; continue; }
      if (c.valid && !c.valid[i]) ok = false;
      l += c.lens[i];
    }
    out_len[i] = ok ? l : 0;
    out_valid[i] = ok;
  }
}

__global__ void concat_write_kernel(const ConcatPart* __restrict__ parts, int32_t k, int64_t n,
                                    const int64_t* __restrict__ off, const uint8_t* __restrict__ ok,
                                    uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!ok[i]) continue;
    uint8_t* d = dst + off[i];
    for (int32_t p = 0; p < k; ++p) {
      const ConcatPart& c = parts[p];
      const uint8_t* s = c.is_lit ? c.lit : c.arena + c.starts[i];
      const int32_t l = c.is_lit ? c.lit_len : c.lens[i];
      for (int32_t q = 0; q < l; ++q) d[q] = s[q];
      d += l;
    }
  }
}

// concat_ws(sep, part_0, …): null parts are skipped and the separator goes between the parts that remain.
__global__ void concat_ws_len_kernel(const ConcatPart* __restrict__ parts, int32_t k, int64_t n, int32_t sl,
                                     int64_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t l = 0;
    int32_t m = 0;
    for (int32_t p = 0; p < k; ++p) {
      const ConcatPart& c = parts[p];
      if (!c.is_lit && c.valid && !c.valid[i]) continue;
      l += c.is_lit ? c.lit_len : c.lens[i];
      ++m;
    }
    out_len[i] = l + (m > 1 ? (int64_t)(m - 1) * sl : 0);
  }
}

__global__ void concat_ws_write_kernel(const ConcatPart* __restrict__ parts, int32_t k, int64_t n,
                                       const uint8_t* __restrict__ sep, int32_t sl, const int64_t* __restrict__ off,
                                       uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t* d = dst + off[i];
    bool first = true;
    for (int32_t p = 0; p < k; ++p) {
      const ConcatPart& c = parts[p];
      if (!c.is_lit && c.valid && !c.valid[i]) continue;
      if (!first)
        for (int32_t q = 0; q < sl; ++q) *d++ = sep[q];
      first = false;
      const uint8_t* s = c.is_lit ? c.lit : c.arena + c.starts[i];
      const int32_t l = c.is_lit ? c.lit_len : c.lens[i];
      for (int32_t q = 0; q < l; ++q) d[q] = s[q];
      d += l;
    }
  }
}

DXA_API int dxa_concat_ws_len(const void* parts, int32_t k, int64_t n, int32_t sl, int64_t* out_len, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(concat_ws_len_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st,
                     (const ConcatPart*)parts, k, n, sl, out_len);
  return (int)hipGetLastError();
}

DXA_API int dxa_concat_ws_write(const void* parts, int32_t k, int64_t n, const uint8_t* sep, int32_t sl,
                                const int64_t* off, uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(concat_ws_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st,
                     (const ConcatPart*)parts, k, n, sep, sl, off, dst);
  return (int)hipGetLastError();
}

__device__ __forceinline__ int i64_digits(int64_t v) {
  uint64_t u = v < 0 ? (0ull - (uint64_t)v) : (uint64_t)v;
  int d = 1;
  while (u >= 10) { u /= 10; ++d; }
  return d + (v < 0);
}

__global__ void i64_len_kernel(const int64_t* __restrict__ v, int64_t n, int64_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out_len[i] = i64_digits(v[i]);
}

__global__ void i64_write_kernel(const int64_t* __restrict__ v, int64_t n, const int64_t* __restrict__ off,
                                 uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = v[i];
    const int nd = i64_digits(x);
    uint8_t* d = dst + off[i];
    uint64_t u = x < 0 ? (0ull - (uint64_t)x) : (uint64_t)x;
    int p = nd - 1;
    do { d[p--] = (uint8_t)('0' + u % 10); u /= 10; } while (u);
    if (x < 0) d[0] = '-';
  }
}

// CAST(long AS STRING) into fixed 24-byte slots (an int64 prints in at most 20 bytes): one launch, no length pass,
// no scan and no host read of the total size.
__global__ void i64_slot_kernel(const int64_t* __restrict__ v, int64_t n, uint8_t* __restrict__ dst,
                                int64_t* __restrict__ starts, int32_t* __restrict__ lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = v[i];
    const int nd = i64_digits(x);
    uint8_t* d = dst + i * 24;
    uint64_t u = x < 0 ? (0ull - (uint64_t)x) : (uint64_t)x;
    int p = nd - 1;
    do { d[p--] = (uint8_t)('0' + u % 10); u /= 10; } while (u);
    if (x < 0) d[0] = '-';
    starts[i] = i * 24;
    lens[i] = nd;
  }
}

// mode 0: lower, 1: upper (ASCII; bytes ≥ 0x80 untouched, matching Spark for ASCII data)
__global__ void case_map_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                const int32_t* __restrict__ lens, int64_t n, const int64_t* __restrict__ off,
                                uint8_t* __restrict__ dst, int mode) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    uint8_t* d = dst + off[i];
    const int32_t l = lens[i];
    for (int32_t k = 0; k < l; ++k) {
      uint8_t c = s[k];
      if (mode == 0 && c >= 'A' && c <= 'Z') c += 32;
      if (mode == 1 && c >= 'a' && c <= 'z') c -= 32;
      d[k] = c;
    }
  }
}

// stringToTimestamp over a string column (dxa_ts.h has the grammar)
__global__ void str_to_ts_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                 const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                                 int64_t* __restrict__ out, uint8_t* __restrict__ out_valid) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t us = 0;
    const bool ok = !(valid && !valid[r]) && dxa::string_to_ts(arena + starts[r], lens[r], us);
    out[r] = ok ? us : 0;
    out_valid[r] = ok;
  }
}

}  // namespace

DXA_API int dxa_str_cmp_lit(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                            const uint8_t* lit, int32_t lit_len, int32_t op, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_cmp_lit_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, lit, lit_len, op, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_eq_col(const uint8_t* aa, const int64_t* as, const int32_t* al, const uint8_t* ba,
                           const int64_t* bs, const int32_t* bl, int64_t n, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_eq_col_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, aa, as, al, ba, bs,
                     bl, n, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_cmp_col(const uint8_t* aa, const int64_t* as, const int32_t* al, const uint8_t* ba,
                            const int64_t* bs, const int32_t* bl, int64_t n, int32_t op, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  if (op < 2 || op > 5) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_cmp_col_kernel, dim3(dxa::grid_stride_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, aa, as,
                     al, ba, bs, bl, n, op, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_gather(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           const int64_t* dst_off, uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_gather_lane_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st,
                       arena, starts, lens, n, dst_off, dst);
  return (int)hipGetLastError();
}

// split(str, literal delimiter) → K slot views into the same arena (no bytes move).  Pass 1 counts each row's
// parts (delimiters + 1; Spark keeps empty and trailing-empty parts), pass 2 writes slot j's start / length for
// j < count and length -1 (absent) for the rest.  One lane per row: strings in DataX events are short.
__device__ __forceinline__ bool delim_at(const uint8_t* p, const uint8_t* d, int32_t dl) {
  for (int32_t k = 0; k < dl; ++k)
    if (p[k] != d[k]) return false;
  return true;
}

__global__ void str_split_count_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                       const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ d,
                                       int32_t dl, int32_t* __restrict__ count) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int32_t c = 1;
    for (int32_t k = 0; k + dl <= l;) {
      if (delim_at(s + k, d, dl)) { ++c; k += dl; } else { ++k; }
    }
    count[i] = c;
  }
}

__global__ void str_split_write_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                       const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ d,
                                       int32_t dl, int32_t K, int64_t* __restrict__ out_starts,
                                       int32_t* __restrict__ out_lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s0 = starts[i];
    const uint8_t* s = arena + s0;
    const int32_t l = lens[i];
    int32_t j = 0, b = 0;
    for (int32_t k = 0; k + dl <= l && j < K;) {
      if (delim_at(s + k, d, dl)) {
        out_starts[(int64_t)j * n + i] = s0 + b;
        out_lens[(int64_t)j * n + i] = k - b;
        ++j;
        k += dl;
        b = k;
      } else {
        ++k;
      }
    }
    if (j < K) {
      out_starts[(int64_t)j * n + i] = s0 + b;
      out_lens[(int64_t)j * n + i] = l - b;
      ++j;
    }
    for (; j < K; ++j) {
      out_starts[(int64_t)j * n + i] = s0;
      out_lens[(int64_t)j * n + i] = -1;
    }
  }
}

DXA_API int dxa_str_split_count(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                                const uint8_t* d, int32_t dl, int32_t* count, void* st) {
  if (n <= 0) return 0;
  if (dl <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_split_count_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, d, dl, count);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_split_write(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                                const uint8_t* d, int32_t dl, int32_t K, int64_t* out_starts, int32_t* out_lens,
                                void* st) {
  if (n <= 0 || K <= 0) return 0;
  if (dl <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_split_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, d, dl, K, out_starts, out_lens);
  return (int)hipGetLastError();
}

// date_format(ts, pattern) for fixed-width patterns: every row renders to exactly L bytes, so the output arena is
// n*L with no length pass and no host synchronisation.  Ops (int32): low byte = field code, bits 8.. = argument
// (literal: offset << 8 | len << 24 into `lits`).  Codes: 0 literal, 1 yyyy, 2 yy, 3 MM, 4 dd, 5 HH, 6 hh, 7 mm,
// 8 ss, 9 SSS, 10 SSSSSS, 11 a (AM/PM), 12 MMM (Jan…), 13 EEE (Mon…), 14 D (day of year, 3 digits: DDD).
__device__ __forceinline__ void put_num(uint8_t* o, int64_t v, int w) {
  for (int k = w - 1; k >= 0; --k) {
    o[k] = (uint8_t)('0' + (v % 10));
    v /= 10;
  }
}

__global__ void ts_format_kernel(const int64_t* __restrict__ us, int64_t n, const int32_t* __restrict__ ops,
                                 int32_t nops, const uint8_t* __restrict__ lits, int32_t L, uint8_t* __restrict__ out) {
  const char* mon = "JanFebMarAprMayJunJulAugSepOctNovDec";
  const char* dow = "MonTueWedThuFriSatSun";
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = us[i];
    int64_t days = t >= 0 ? t / 86400000000ll : -((-t + 86400000000ll - 1) / 86400000000ll);
    const int64_t rem = t - days * 86400000000ll;                    // [0, 1 day) in µs
    const int64_t hh = rem / 3600000000ll, mi = (rem / 60000000ll) % 60, ss = (rem / 1000000ll) % 60;
    const int64_t frac = rem % 1000000ll;
    const int64_t wd = ((days % 7) + 7 + 3) % 7;                     // 0 = Monday (1970-01-01 was a Thursday)
    // civil from days (Hinnant)
    const int64_t z = days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int64_t d = doy - (153 * mp + 2) / 5 + 1;
    const int64_t m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) ++y;
    const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
    const int cum[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
    const int64_t yday = cum[m - 1] + d + (leap && m > 2 ? 1 : 0);
    uint8_t* o = out + i * L;
    for (int32_t k = 0; k < nops; ++k) {
      const int32_t op = ops[k], code = op & 0xff;
      switch (code) {
        case 0: {
          const int32_t off = (op >> 8) & 0xffff, len = (op >> 24) & 0xff;
          for (int32_t b = 0; b < len; ++b) o[b] = lits[off + b];
          o += len;
          break;
        }
        case 1: put_num(o, y < 0 ? 0 : y, 4); o += 4; break;
        case 2: put_num(o, (y % 100 + 100) % 100, 2); o += 2; break;
        case 3: put_num(o, m, 2); o += 2; break;
        case 4: put_num(o, d, 2); o += 2; break;
        case 5: put_num(o, hh, 2); o += 2; break;
        case 6: put_num(o, (hh % 12) == 0 ? 12 : hh % 12, 2); o += 2; break;
        case 7: put_num(o, mi, 2); o += 2; break;
        case 8: put_num(o, ss, 2); o += 2; break;
        case 9: put_num(o, frac / 1000, 3); o += 3; break;
        case 10: put_num(o, frac, 6); o += 6; break;
        case 11: o[0] = hh < 12 ? 'A' : 'P'; o[1] = 'M'; o += 2; break;
        case 12: for (int b = 0; b < 3; ++b) o[b] = (uint8_t)mon[(m - 1) * 3 + b]; o += 3; break;
        case 13: for (int b = 0; b < 3; ++b) o[b] = (uint8_t)dow[wd * 3 + b]; o += 3; break;
        case 14: put_num(o, yday, 3); o += 3; break;
        default: break;
      }
    }
  }
}

DXA_API int dxa_ts_format(const int64_t* us, int64_t n, const int32_t* ops, int32_t nops, const uint8_t* lits,
                          int32_t L, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ts_format_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, us, n, ops, nops,
                     lits, L, out);
  return (int)hipGetLastError();
}

// ---- character-level string functions (UTF-8 aware: a character starts at every byte that is not 10xxxxxx) ----
__device__ __forceinline__ bool utf8_lead(uint8_t b) { return (b & 0xC0) != 0x80; }

// Byte offset of character k (0-based) in s[0, l); l if the string has fewer characters.
__device__ __forceinline__ int32_t char_to_byte(const uint8_t* s, int32_t l, int64_t k) {
  if (k <= 0) return 0;
  int64_t c = -1;
  for (int32_t i = 0; i < l; ++i) {
    if (utf8_lead(s[i]) && ++c == k) return i;
  }
  return l;
}

__device__ __forceinline__ int32_t num_chars(const uint8_t* s, int32_t l) {
  int32_t c = 0;
  for (int32_t i = 0; i < l; ++i) c += utf8_lead(s[i]);
  return c;
}

// substring(str, pos, len) with Spark's UTF8String.substringSQL semantics, as a view (new start / length).
// len == INT64_MAX: to the end.  pos / len may be per-row (non-null pointer) or constants.
__global__ void str_substr_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, int64_t n, const int64_t* __restrict__ pos_col,
                                  int64_t pos_c, const int64_t* __restrict__ len_col, int64_t len_c,
                                  int64_t* __restrict__ out_starts, int32_t* __restrict__ out_lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    const int64_t pos = pos_col ? pos_col[i] : pos_c;
    const int64_t length = len_col ? len_col[i] : len_c;
    int64_t nch = -1;                                      // computed only when needed
    int64_t start = pos > 0 ? pos - 1 : 0;
    if (pos < 0) { nch = num_chars(s, l); start = nch + pos; }
    int64_t end;
    if (length == INT64_MAX) end = INT64_MAX;
    else end = start + length;
    if (start < 0) start = 0;
    int32_t b0 = 0, b1 = 0;
    if (start < end) {
      b0 = char_to_byte(s, l, start);
      b1 = end == INT64_MAX ? l : char_to_byte(s, l, end);
      if (b1 < b0) b1 = b0;
    }
    out_starts[i] = starts[i] + b0;
    out_lens[i] = b1 - b0;
  }
}

// trim / ltrim / rtrim of ASCII spaces (mode bit 0: left, bit 1: right), as a view.
__global__ void str_trim_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                const int32_t* __restrict__ lens, int64_t n, int32_t mode,
                                int64_t* __restrict__ out_starts, int32_t* __restrict__ out_lens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    int32_t a = 0, b = lens[i];
    if (mode & 1) while (a < b && s[a] == ' ') ++a;
    if (mode & 2) while (b > a && s[b - 1] == ' ') --b;
    out_starts[i] = starts[i] + a;
    out_lens[i] = b - a;
  }
}

__global__ void str_numchars_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                    const int32_t* __restrict__ lens, int64_t n, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = num_chars(arena + starts[i], lens[i]);
}

// locate(needle, str, start_char): 1-based character position of the first occurrence at or after character
// start_char (1-based; < 1 → 0 result), 0 when absent.  instr(str, needle) = locate(needle, str, 1).
__device__ __forceinline__ int32_t utf8_len(uint8_t b) {
  return b < 0x80 ? 1 : (b & 0xE0) == 0xC0 ? 2 : (b & 0xF0) == 0xE0 ? 3 : (b & 0xF8) == 0xF0 ? 4 : 1;
}

// (UTF8String.indexOf(needle, from - 1) + 1, as Spark's StringLocate; an empty needle is found at 1)
__global__ void str_locate_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ d,
                                  int32_t dl, int64_t from, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int64_t r = 0;
    if (from >= 1) {
      if (dl == 0) {
        r = 1;
      } else {
        int32_t b = 0;
        int64_t c = 0;
        while (b < l && c < from - 1) { b += utf8_len(s[b]); ++c; }
        while (b + dl <= l) {
          if (delim_at(s + b, d, dl)) { r = c + 1; break; }
          b += utf8_len(s[b]);
          ++c;
        }
      }
    }
    out[i] = r;
  }
}

// replace(str, search, rep) with literal search / replacement: pass 1 writes each row's output length, pass 2
// (after the host's exclusive scan) writes the bytes.  Non-overlapping, left to right (String.replace).
__global__ void str_replace_len_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                       const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ d,
                                       int32_t dl, int32_t rl, int64_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int64_t o = 0;
    for (int32_t k = 0; k < l;) {
      if (k + dl <= l && delim_at(s + k, d, dl)) { o += rl; k += dl; } else { ++o; ++k; }
    }
    out_len[i] = o;
  }
}

__global__ void str_replace_write_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                         const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ d,
                                         int32_t dl, const uint8_t* __restrict__ rep, int32_t rl,
                                         const int64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* o = dst + off[i];
    for (int32_t k = 0; k < l;) {
      if (k + dl <= l && delim_at(s + k, d, dl)) {
        for (int32_t j = 0; j < rl; ++j) *o++ = rep[j];
        k += dl;
      } else {
        *o++ = s[k++];
      }
    }
  }
}

DXA_API int dxa_str_substr(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           const int64_t* pos_col, int64_t pos_c, const int64_t* len_col, int64_t len_c,
                           int64_t* out_starts, int32_t* out_lens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_substr_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, pos_col, pos_c, len_col, len_c, out_starts, out_lens);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_trim(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n, int32_t mode,
                         int64_t* out_starts, int32_t* out_lens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_trim_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, n,
                     mode, out_starts, out_lens);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_numchars(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                             int64_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_numchars_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_locate(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           const uint8_t* d, int32_t dl, int64_t from, int64_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_locate_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, d, dl, from, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_replace_len(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                                const uint8_t* d, int32_t dl, int32_t rl, int64_t* out_len, void* st) {
  if (n <= 0) return 0;
  if (dl <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_replace_len_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, d, dl, rl, out_len);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_replace_write(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                                  const uint8_t* d, int32_t dl, const uint8_t* rep, int32_t rl, const int64_t* off,
                                  uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  if (dl <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_replace_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, d, dl, rep, rl, off, dst);
  return (int)hipGetLastError();
}

// CAST(string AS BIGINT | INT | DOUBLE) with Spark's non-ANSI semantics: surrounding whitespace (<= ' ') ignored;
// integers: [+-]digits[.digits] (the fraction truncates; no exponent), out of range → null; doubles: decimal with
// optional exponent, or inf / infinity / nan (any case, optional sign).  mode 0 long, 1 int, 2 double.
__device__ __forceinline__ bool ci_eq(const uint8_t* s, int32_t l, const char* w) {
  int32_t k = 0;
  for (; w[k]; ++k)
    if (k >= l || (s[k] | 0x20) != w[k]) return false;
  return k == l;
}

__global__ void str_to_num_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                                  int32_t mode, int64_t* __restrict__ out, uint8_t* __restrict__ out_ok) {
  const double kP10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                           1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = 0;
    out_ok[i] = 0;
    if (valid && !valid[i]) continue;
    const uint8_t* s = arena + starts[i];
    int32_t a = 0, b = lens[i];
    while (a < b && s[a] <= ' ') ++a;
    while (b > a && s[b - 1] <= ' ') --b;
    if (a >= b) continue;
    bool neg = false;
    int32_t p = a;
    if (s[p] == '+' || s[p] == '-') { neg = s[p] == '-'; ++p; }
    if (mode == 2) {
      const int32_t l = b - p;
      if (ci_eq(s + p, l, "inf") || ci_eq(s + p, l, "infinity")) {
        out[i] = __double_as_longlong(neg ? -__builtin_inf() : __builtin_inf());
        out_ok[i] = 1;
        continue;
      }
      if (ci_eq(s + p, l, "nan") && p == a) {
        out[i] = __double_as_longlong(__builtin_nan(""));
        out_ok[i] = 1;
        continue;
      }
    }
    uint64_t mant = 0, tail = 0;                          // first 19 significant digits, the next 19
    int nd = 0, exp10 = 0, digits = 0, nt = 0;
    bool lost = false;
    for (; p < b && s[p] - '0' < 10u; ++p, ++digits) {
      if (nd < 19) { mant = mant * 10 + (s[p] - '0'); if (mant) ++nd; }
      else { ++exp10; lost = true; if (nt < 19) { tail = tail * 10 + (s[p] - '0'); ++nt; } }
    }
    int fdigits = 0;
    if (p < b && s[p] == '.') {
      ++p;
      for (; p < b && s[p] - '0' < 10u; ++p, ++fdigits) {
        if (mode != 2) continue;
        if (nd < 19) { mant = mant * 10 + (s[p] - '0'); if (mant) ++nd; --exp10; }
        else if (nt < 19) { tail = tail * 10 + (s[p] - '0'); ++nt; }
      }
    }
    if (digits + fdigits == 0) continue;
    if (mode == 2 && p < b && (s[p] | 0x20) == 'e') {
      ++p;
      bool eneg = false;
      if (p < b && (s[p] == '+' || s[p] == '-')) { eneg = s[p] == '-'; ++p; }
      int e = 0, ed = 0;
      for (; p < b && s[p] - '0' < 10u; ++p, ++ed)
        if (e < 100000) e = e * 10 + (s[p] - '0');
      if (!ed) continue;
      exp10 += eneg ? -e : e;
    }
    if (p != b) continue;                                 // trailing garbage
    if (mode == 2) {
      double d = (double)mant;
      if (mant == 0) d = 0.0;
      else if (tail == 0 && mant < (1ull << 53) && exp10 >= 0 && exp10 <= 22) d = d * kP10[exp10];
      else if (tail == 0 && mant < (1ull << 53) && exp10 < 0 && exp10 >= -22) d = d / kP10[-exp10];
      else if (exp10 > DXA_POW10_DD_MAX) d = __builtin_inf();
      else if (exp10 < DXA_POW10_DD_MIN) d = 0.0;
      else d = dxa_decimal_to_double(mant, exp10, tail, nt);
      out[i] = __double_as_longlong(neg ? -d : d);
      out_ok[i] = 1;
      continue;
    }
    if (lost) continue;                                   // more than 19 integer digits
    const uint64_t lim = mode == 1 ? (neg ? 2147483648ull : 2147483647ull)
                                   : (neg ? 9223372036854775808ull : 9223372036854775807ull);
    if (mant > lim) continue;
    out[i] = neg ? (int64_t)(0ull - mant) : (int64_t)mant;
    out_ok[i] = 1;
  }
}

DXA_API int dxa_str_to_num(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                           int64_t n, int32_t mode, int64_t* out, uint8_t* out_ok, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_to_num_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, n, mode, out, out_ok);
  return (int)hipGetLastError();
}

// General LIKE on the device.  Pattern tokens (int16): 0..255 a literal byte, 256 '_' (one UTF-8 character),
// 257 '%' (any sequence); escapes are resolved by the host.  Greedy match with one backtrack point (the last '%'):
// linear in practice, exact for LIKE's two wildcards.
__global__ void str_like_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                const int32_t* __restrict__ lens, int64_t n, const int16_t* __restrict__ tok,
                                int32_t m, uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int32_t si = 0, pi = 0, star_p = -1, star_s = 0;
    bool ok = true;
    while (si < l) {
      const int32_t t = pi < m ? tok[pi] : -1;
      if (t == 256) { si += utf8_len(s[si]); ++pi; continue; }
      if (t >= 0 && t < 256 && s[si] == (uint8_t)t) { ++si; ++pi; continue; }
      if (t == 257) { star_p = pi++; star_s = si; continue; }
      if (star_p >= 0) {
        pi = star_p + 1;
        star_s += utf8_len(s[star_s]);
        si = star_s;
        continue;
      }
      ok = false;
      break;
    }
    if (ok) {
      while (pi < m && tok[pi] == 257) ++pi;
      ok = pi == m && si <= l;
    }
    out[i] = ok;
  }
}

DXA_API int dxa_str_like(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                         const int16_t* tok, int32_t m, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_like_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, tok, m, out);
  return (int)hipGetLastError();
}

// regexp_extract / regexp_replace: a backtracking program (regex_vm.py) per row, Java's match choice (leftmost
// start; SPLIT x,y tries x first).  Backtrack stack and step budget are bounded; a row that exceeds either gets
// status 1 and the host recomputes the column.
constexpr int kRxStack = 64;
constexpr int kRxBudget = 1 << 16;
constexpr int kRxCaps = 32;                // 2 × (9 groups + 1) captures, then loop position registers

struct RxArgs {
  const uint8_t* arena; const int64_t* starts; const int32_t* lens; int64_t n;
  const int4* prog; const uint32_t* sets;
  int32_t mode;                       // 0 extract group, 1 replace: lengths, 2 replace: write
  int32_t group;
  const int32_t* rep; int32_t nrep;   // replacement tokens: byte, or -1-k for group k
  int64_t* out_start; int32_t* out_len; const int64_t* out_off; uint8_t* out; uint8_t* status;
  const uint8_t* hit;                 // optional RLIKE prefilter (the DFA): rows without a match skip the search
  int32_t nprog, nsets;
};

__device__ __forceinline__ bool rx_bit(const uint32_t* sets, int k, uint32_t c) {
  return (sets[k * 8 + (c >> 5)] >> (c & 31)) & 1;
}

// 1 matched (cap filled), 0 no match from this start, -1 over budget
__device__ int rx_match_at(const RxArgs& a, const uint8_t* s, int32_t len, int32_t start, int32_t* cap, int& steps) {
  int32_t stk[3 * kRxStack];          // (kind << 24 | pc or capture slot, sp or old value) + spare
  int top = 0;
  for (int k = 0; k < kRxCaps; ++k) cap[k] = -1;
  stk[0] = 0; stk[1] = start; top = 1;
  while (top > 0) {
    --top;
    const int32_t tag = stk[2 * top];
    if (tag < 0) { cap[-1 - tag] = stk[2 * top + 1]; continue; }            // restore a capture
    int32_t pc = tag, sp = stk[2 * top + 1];
    while (true) {
      if (++steps > kRxBudget) return -1;
      const int4 in = a.prog[pc];
      bool ok = true;
      switch (in.x) {
        case 0:                                   // CHAR
          ok = sp < len && s[sp] == (uint8_t)in.y; sp += ok; ++pc; break;
        case 1:                                   // SET
          ok = sp < len && s[sp] < 128 && rx_bit(a.sets, in.y, s[sp]); sp += ok; ++pc; break;
        case 2: {                                 // ANY: one code point, not a line terminator
          if (sp >= len) { ok = false; break; }
          const uint8_t c = s[sp];
          const int32_t u = utf8_len(c);
          if (c == '\n' || c == '\r') ok = false;
          else if (c == 0xC2 && sp + 1 < len && s[sp + 1] == 0x85) ok = false;
          else if (c == 0xE2 && sp + 2 < len && s[sp + 1] == 0x80 && (s[sp + 2] == 0xA8 || s[sp + 2] == 0xA9)) ok = false;
          sp += (sp + u <= len) ? u : len - sp; ++pc; break;
        }
        case 3: {                                 // NOTSET: one code point outside an ASCII set
          if (sp >= len) { ok = false; break; }
          const uint8_t c = s[sp];
          if (c < 128) { ok = !rx_bit(a.sets, in.y, c); sp += 1; }
          else { const int32_t u = utf8_len(c); sp += (sp + u <= len) ? u : len - sp; }
          ++pc; break;
        }
        case 4:                                   // SPLIT: try a, remember b
          if (top >= kRxStack) return -1;
          stk[2 * top] = in.z; stk[2 * top + 1] = sp; ++top; pc = in.y; break;
        case 5: pc = in.y; break;                 // JMP
        case 6:                                   // SAVE
          if (top >= kRxStack) return -1;
          stk[2 * top] = -1 - in.y; stk[2 * top + 1] = cap[in.y]; ++top;
          cap[in.y] = sp; ++pc; break;
        case 7: ok = sp == 0; ++pc; break;        // BOL
        case 8: {                                 // EOL: Java $ (Pattern.Dollar) — end, or before a final
          const int64_t r = len - sp;             // \r\n, \n (not after \r), \r, U+0085, U+2028, U+2029
          ok = r == 0 ||
               (r == 1 && (s[sp] == '\n' ? !(sp > 0 && s[sp - 1] == '\r') : s[sp] == '\r')) ||
               (r == 2 && ((s[sp] == '\r' && s[sp + 1] == '\n') || (s[sp] == 0xC2 && s[sp + 1] == 0x85))) ||
               (r == 3 && s[sp] == 0xE2 && s[sp + 1] == 0x80 && (s[sp + 2] == 0xA8 || s[sp + 2] == 0xA9));
          ++pc;
          break;
        }
        case 10: pc = sp == cap[in.y] ? in.w : in.z; break;                          // LOOP: no progress → leave
        case 9: return 1;                         // MATCH
        default: return -1;
      }
      if (!ok) break;
    }
  }
  return 0;
}

// leftmost match starting at or after `from` (code-point boundaries): 1 found, 0 none, -1 over budget
__device__ int rx_find(const RxArgs& a, const uint8_t* s, int32_t len, int32_t from, int32_t* cap, int& steps) {
  for (int32_t st = from; st <= len; ++st) {
    if (st < len && (s[st] & 0xC0) == 0x80) continue;                    // inside a code point
    const int r = rx_match_at(a, s, len, st, cap, steps);
    if (r != 0) return r;
  }
  return 0;
}

constexpr int kRxLdsInts = 4096;      // program + bitmaps staged in LDS when they fit (16 KB)

__global__ void __launch_bounds__(256) str_regex_kernel(RxArgs a) {
  __shared__ int32_t rx_sh[kRxLdsInts];
  const int words = a.nprog * 4 + a.nsets * 8;
  if (words <= kRxLdsInts) {
    for (int k = threadIdx.x; k < a.nprog * 4; k += blockDim.x) rx_sh[k] = ((const int32_t*)a.prog)[k];
    for (int k = threadIdx.x; k < a.nsets * 8; k += blockDim.x) rx_sh[a.nprog * 4 + k] = (int32_t)a.sets[k];
    __syncthreads();
    a.prog = (const int4*)rx_sh;
    a.sets = (const uint32_t*)(rx_sh + a.nprog * 4);
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = a.arena + a.starts[i];
    const int32_t len = a.lens[i];
    int32_t cap[kRxCaps];
    int steps = 0;
    uint8_t bad = 0;
    const bool skip = a.hit != nullptr && !a.hit[i];
    if (a.mode == 0) {
      const int r = skip ? 0 : rx_find(a, s, len, 0, cap, steps);
      int32_t b = 0, e = 0;
      if (r == 1 && cap[2 * a.group] >= 0 && cap[2 * a.group + 1] >= 0) { b = cap[2 * a.group]; e = cap[2 * a.group + 1]; }
      bad = r < 0;
      a.out_start[i] = a.starts[i] + b;
      a.out_len[i] = e - b;
    } else {
      uint8_t* o = a.mode == 2 ? a.out + a.out_off[i] : nullptr;
      int64_t olen = 0;
      int32_t pos = 0, last = 0;
      while (!skip && pos <= len) {
        const int r = rx_find(a, s, len, pos, cap, steps);
        if (r < 0) { bad = 1; break; }
        if (r == 0) break;
        const int32_t ms = cap[0], me = cap[1];
        if (o) for (int32_t k = last; k < ms; ++k) o[olen + k - last] = s[k];
        olen += ms - last;
        for (int32_t t = 0; t < a.nrep; ++t) {
          const int32_t tk = a.rep[t];
          if (tk >= 0) { if (o) o[olen] = (uint8_t)tk; ++olen; continue; }
          const int32_t g = -1 - tk, gb = cap[2 * g], ge = cap[2 * g + 1];
          if (gb < 0 || ge < 0) continue;
          if (o) for (int32_t k = gb; k < ge; ++k) o[olen + k - gb] = s[k];
          olen += ge - gb;
        }
        last = me;
        pos = me > ms ? me : me + (me < len ? utf8_len(s[me]) : 1);
      }
      if (!bad) {
        if (o) for (int32_t k = last; k < len; ++k) o[olen + k - last] = s[k];
        olen += len - last;
      }
      if (a.mode == 1) a.out_len[i] = bad ? 0 : (int32_t)olen;
    }
    a.status[i] = bad;
  }
}

DXA_API int dxa_str_regex(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                          const int32_t* prog, int32_t nprog, const int32_t* sets, int32_t nsets, int32_t mode,
                          int32_t group, const int32_t* rep, int32_t nrep, int64_t* out_start, int32_t* out_len,
                          const int64_t* out_off, uint8_t* out, uint8_t* status, const uint8_t* hit, void* st) {
  if (n <= 0) return 0;
  if (mode < 0 || mode > 2 || group < 0 || group > 9) return (int)hipErrorInvalidValue;
  RxArgs a{arena, starts, lens, n, (const int4*)prog, (const uint32_t*)sets, mode, group, rep, nrep,
           out_start, out_len, out_off, out, status, hit, nprog, nsets};
  hipLaunchKernelGGL(str_regex_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

// RLIKE on the device: a byte-level DFA (regex_dfa.py) over symbol classes, run from BOS through the bytes to
// EOS.  blob = [class of each symbol (258) | next-state table (states × classes)], staged in LDS; a table entry with
// bit 15 set leads to a terminal state (dead, or accepting — accepting states absorb), so a row stops as soon as
// its answer is known.
__global__ void __launch_bounds__(256) str_rlike_kernel(const uint8_t* __restrict__ arena,
                                                        const int64_t* __restrict__ starts,
                                                        const int32_t* __restrict__ lens, int64_t n,
                                                        const int16_t* __restrict__ blob, int32_t words,
                                                        int32_t ncls, int32_t start, uint8_t* __restrict__ out) {
  extern __shared__ int16_t dfa_sh[];
  for (int k = threadIdx.x; k < words; k += blockDim.x) dfa_sh[k] = blob[k];
  __syncthreads();
  const int16_t* cls = dfa_sh;
  const int16_t* tab = dfa_sh + 258;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int32_t e = tab[start * ncls + cls[256]];
    for (int32_t p = 0; e >= 0 && p < l; ++p) e = tab[e * ncls + cls[s[p]]];
    if (e >= 0) e = tab[e * ncls + cls[257]];
    out[i] = e < 0 && (e & 0x7fff) != 0;
  }
}

DXA_API int dxa_str_rlike(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                          const int16_t* blob, int32_t words, int32_t ncls, int32_t start, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  if (words > 258 + 16384 || ncls <= 0 || ncls > 258) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(str_rlike_kernel, dim3(dxa_blocks(n, 256, 1024)), dim3(256), (size_t)words * 2, (hipStream_t)st,
                     arena, starts, lens, n, blob, words, ncls, start, out);
  return (int)hipGetLastError();
}

// parts: host array of k StrPart descriptors (row0 relative to the first part); launches in groups of kMaxStrParts.
DXA_API int dxa_str_gather_parts(const void* parts, int32_t k, void* st) {
  const StrPart* ps = (const StrPart*)parts;
  for (int32_t g = 0; g < k; g += kMaxStrParts) {
    const int32_t kk = k - g < kMaxStrParts ? k - g : kMaxStrParts;
    StrParts a{};
    const int64_t base = ps[g].row0;
    for (int32_t j = 0; j < kk; ++j) {
      a.p[j] = ps[g + j];
      a.p[j].row0 -= base;
    }
    a.k = kk;
    // the group ends where the next part begins; the caller appends an end sentinel (row0 = total) after part k-1
    a.total = ps[g + kk].row0 - base;
    if (a.total <= 0) continue;
    hipLaunchKernelGGL(str_gather_parts_kernel, dim3((unsigned)((a.total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)st, a);
  }
  return (int)hipGetLastError();
}

DXA_API int dxa_str_part_size() { return (int)sizeof(StrPart); }

// parts: device array of ConcatPart (k entries) prepared by the host.
DXA_API int dxa_concat_len(const void* parts, int32_t k, int64_t n, int64_t* out_len, uint8_t* out_valid, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(concat_len_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st,
                     (const ConcatPart*)parts, k, n, out_len, out_valid);
  return (int)hipGetLastError();
}

DXA_API int dxa_concat_write(const void* parts, int32_t k, int64_t n, const int64_t* off, const uint8_t* ok,
                             uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(concat_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st,
                     (const ConcatPart*)parts, k, n, off, ok, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_concat_part_size() { return (int)sizeof(ConcatPart); }

DXA_API int dxa_i64_to_str_len(const int64_t* v, int64_t n, int64_t* out_len, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(i64_len_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, n, out_len);
  return (int)hipGetLastError();
}

DXA_API int dxa_i64_to_str_write(const int64_t* v, int64_t n, const int64_t* off, uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(i64_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, n, off, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_i64_to_str_slots(const int64_t* v, int64_t n, uint8_t* dst, int64_t* starts, int32_t* lens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(i64_slot_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, n, dst, starts,
                     lens);
  return (int)hipGetLastError();
}

DXA_API int dxa_case_map(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                         const int64_t* off, uint8_t* dst, int mode, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(case_map_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, n,
                     off, dst, mode);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_to_ts(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                          int64_t n, int64_t* out, uint8_t* out_valid, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_to_ts_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, n, out, out_valid);
  return (int)hipGetLastError();
}

// Input normaliser byte map (kernel K2: e.g. control characters → '#', RemoveInvalidChars.scala:12-17): every byte
// of the raw batch goes through a 256-entry table held in LDS; 16 bytes per lane per iteration (dwordx4 loads and
// stores), grid-stride so one launch covers any batch size.
__global__ __launch_bounds__(256) void byte_map_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int64_t n, const uint8_t* __restrict__ map) {
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = map[threadIdx.x];
  __syncthreads();
  const int64_t nvec = n / 16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    uint4 w = reinterpret_cast<const uint4*>(src)[v];
    uint32_t* p = reinterpret_cast<uint32_t*>(&w);
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = p[k];
      p[k] = (uint32_t)lut[x & 0xff] | ((uint32_t)lut[(x >> 8) & 0xff] << 8) | ((uint32_t)lut[(x >> 16) & 0xff] << 16) |
             ((uint32_t)lut[x >> 24] << 24);
    }
    reinterpret_cast<uint4*>(dst)[v] = w;
  }
  for (int64_t i = nvec * 16 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = lut[src[i]];
}

DXA_API int dxa_byte_map(const uint8_t* src, uint8_t* dst, int64_t n, const uint8_t* map, void* st) {
  if (n <= 0) return 0;
  if ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) return -1;      // callers pass 16-B aligned allocations
  int64_t blocks = (n / 16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(byte_map_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)st, src, dst, n, map);
  return (int)hipGetLastError();
}
