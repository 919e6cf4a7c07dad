// Spark string built-ins on device string columns (K10 in SURVEY.md §2.F: user SQL runs in Spark's whole-stage
// codegen on the executors, CommonProcessorFactory.scala:257-275).  Character semantics are UTF-8 code points, as
// Spark's UTF8String: lpad / rpad (UTF8String.lpad/rpad), reverse, repeat, translate, initcap (lower-case, then
// title-case after ' '), substring_index (a view, no bytes move) and levenshtein.
//
// Shape: one lane per row (strings in DataX events are short).  Functions whose output length differs from the
// input run as a length pass, a scan (torch) and a write pass; same-length ones (reverse, initcap) write straight
// into the compacted offsets.  Rows a kernel cannot handle (initcap / levenshtein over non-ASCII, levenshtein over
// long strings) set a flag; the caller then takes the host path for the column.
#include "dxa_common.h"

namespace {

__device__ __forceinline__ bool is_cont(uint8_t c) { return (c & 0xC0) == 0x80; }

__device__ __forceinline__ int32_t num_chars(const uint8_t* s, int32_t l) {
  int32_t n = 0;
  for (int32_t k = 0; k < l; ++k) n += !is_cont(s[k]);
  return n;
}

// byte offset of the first `chars` characters of s (≤ l)
__device__ __forceinline__ int32_t prefix_bytes(const uint8_t* s, int32_t l, int32_t chars) {
  int32_t k = 0, c = 0;
  while (k < l) {
    if (!is_cont(s[k])) {
      if (c == chars) return k;
      ++c;
    }
    ++k;
  }
  return l;
}

struct PadArgs {
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
  int64_t n;
  int64_t target;          // target length in characters
  const uint8_t* pad;      // pad bytes
  int32_t pad_len;         // bytes
  int32_t pad_chars;
  const int32_t* pad_off;  // [pad_chars + 1] byte offset of every pad character
  int32_t left;            // lpad / rpad
};

// bytes of the padded result of row i
__device__ int64_t pad_bytes(const PadArgs& a, int64_t i, int32_t& keep, int32_t& fill_chars) {
  const uint8_t* s = a.arena + a.starts[i];
  const int32_t l = a.lens[i];
  const int32_t nc = num_chars(s, l);
  fill_chars = 0;
  if (a.target <= 0) { keep = 0; return 0; }
  if (nc >= a.target || a.pad_chars == 0) {
    keep = nc >= a.target ? prefix_bytes(s, l, (int32_t)a.target) : l;
    return keep;
  }
  keep = l;
  fill_chars = (int32_t)(a.target - nc);
  const int64_t full = fill_chars / a.pad_chars, part = fill_chars % a.pad_chars;
  return (int64_t)l + full * a.pad_len + a.pad_off[part];
}

__global__ void pad_len_kernel(const PadArgs a, int64_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t keep, fill;
    out_len[i] = pad_bytes(a, i, keep, fill);
  }
}

__device__ __forceinline__ void fill_pad(const PadArgs& a, uint8_t* d, int32_t fill_chars) {
  int64_t w = 0;
  const int32_t full = fill_chars / a.pad_chars, part = fill_chars % a.pad_chars;
  for (int32_t r = 0; r < full; ++r)
    for (int32_t k = 0; k < a.pad_len; ++k) d[w++] = a.pad[k];
  for (int32_t k = 0; k < a.pad_off[part]; ++k) d[w++] = a.pad[k];
}

__global__ void pad_write_kernel(const PadArgs a, const int64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t keep, fill;
    const int64_t total = pad_bytes(a, i, keep, fill);
    const uint8_t* s = a.arena + a.starts[i];
    uint8_t* d = dst + off[i];
    if (a.left) {
      const int64_t padb = total - keep;
      if (fill) fill_pad(a, d, fill);
      for (int32_t k = 0; k < keep; ++k) d[padb + k] = s[k];
    } else {
      for (int32_t k = 0; k < keep; ++k) d[k] = s[k];
      if (fill) fill_pad(a, d + keep, fill);
    }
  }
}

// reverse by characters: same byte length, written straight at the compacted offsets
__global__ void reverse_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                               const int32_t* __restrict__ lens, int64_t n, const int64_t* __restrict__ off,
                               uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* d = dst + off[i];
    int32_t k = 0;
    while (k < l) {
      int32_t e = k + 1;
      while (e < l && is_cont(s[e])) ++e;
      // char [k, e) goes to [l - e, l - k)
      for (int32_t q = k; q < e; ++q) d[l - e + (q - k)] = s[q];
      k = e;
    }
  }
}

__global__ void repeat_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                              const int32_t* __restrict__ lens, int64_t n, int64_t times,
                              const int64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* d = dst + off[i];
    for (int64_t r = 0; r < times; ++r)
      for (int32_t k = 0; k < l; ++k) d[r * l + k] = s[k];
  }
}

__device__ __forceinline__ uint32_t decode_cp(const uint8_t* s, int32_t l, int32_t& k) {
  const uint8_t c = s[k];
  int extra = c < 0x80 ? 0 : c < 0xE0 ? 1 : c < 0xF0 ? 2 : 3;
  uint32_t cp = extra == 0 ? c : extra == 1 ? (c & 0x1F) : extra == 2 ? (c & 0x0F) : (c & 0x07);
  ++k;
  for (int e = 0; e < extra && k < l; ++e, ++k) cp = (cp << 6) | (s[k] & 0x3F);
  return cp;
}

__device__ __forceinline__ int enc_len(uint32_t cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

__device__ __forceinline__ int encode_cp(uint32_t cp, uint8_t* d) {
  if (cp < 0x80) { d[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { d[0] = 0xC0 | (cp >> 6); d[1] = 0x80 | (cp & 0x3F); return 2; }
  if (cp < 0x10000) {
    d[0] = 0xE0 | (cp >> 12); d[1] = 0x80 | ((cp >> 6) & 0x3F); d[2] = 0x80 | (cp & 0x3F); return 3;
  }
  d[0] = 0xF0 | (cp >> 18); d[1] = 0x80 | ((cp >> 12) & 0x3F); d[2] = 0x80 | ((cp >> 6) & 0x3F);
  d[3] = 0x80 | (cp & 0x3F);
  return 4;
}

// translate: from[m] → to[m] (−1: delete); the first occurrence of a character in `from` wins (host dedups)
__device__ __forceinline__ int64_t tr_map(uint32_t cp, const uint32_t* from, const int32_t* to, int32_t m) {
  for (int32_t j = 0; j < m; ++j)
    if (from[j] == cp) return to[j];
  return (int64_t)cp;
}

__global__ void translate_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                 const int32_t* __restrict__ lens, int64_t n, const uint32_t* __restrict__ from,
                                 const int32_t* __restrict__ to, int32_t m, const int64_t* __restrict__ off,
                                 int64_t* __restrict__ out_len, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int64_t w = 0;
    uint8_t* d = off ? dst + off[i] : nullptr;
    int32_t k = 0;
    while (k < l) {
      const uint32_t cp = decode_cp(s, l, k);
      const int64_t r = tr_map(cp, from, to, m);
      if (r < 0) continue;
      if (d) w += encode_cp((uint32_t)r, d + w);
      else w += enc_len((uint32_t)r);
    }
    if (!off) out_len[i] = w;
  }
}

// initcap: lower-case everything, upper-case the first letter of each ' '-separated word (ASCII; a row with a
// non-ASCII byte sets `bad`)
__global__ void initcap_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                               const int32_t* __restrict__ lens, int64_t n, const int64_t* __restrict__ off,
                               uint8_t* __restrict__ dst, int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* d = dst + off[i];
    bool start = true;
    for (int32_t k = 0; k < l; ++k) {
      uint8_t c = s[k];
      if (c >= 0x80) *bad = 1;
      if (c >= 'A' && c <= 'Z') c += 32;
      if (start && c >= 'a' && c <= 'z') c -= 32;
      start = c == ' ';
      d[k] = c;
    }
  }
}

// substring_index(s, delim, count): a view [start, start + len) of the source
__global__ void substring_index_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                       const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ dl,
                                       int32_t dn, int64_t count, int64_t* __restrict__ out_start,
                                       int32_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int64_t st = starts[i];
    int32_t ln = l;
    if (dn == 0 || count == 0) {
      ln = 0;
    } else if (count > 0) {
      int64_t seen = 0;
      for (int32_t k = 0; k + dn <= l; ++k) {
        bool m = true;
        for (int32_t q = 0; q < dn && m; ++q) m = s[k + q] == dl[q];
        if (m && ++seen == count) { ln = k; break; }
      }
    } else {
      int64_t seen = 0;
      for (int32_t k = l - dn; k >= 0; --k) {
        bool m = true;
        for (int32_t q = 0; q < dn && m; ++q) m = s[k + q] == dl[q];
        if (m && ++seen == -count) { st = starts[i] + k + dn; ln = l - k - dn; break; }
      }
    }
    out_start[i] = st;
    out_len[i] = ln;
  }
}

// levenshtein over bytes of ASCII strings up to kLevMax characters (two rolling rows in private memory); other
// rows set `bad`
constexpr int kLevMax = 128;

__global__ void levenshtein_kernel(const uint8_t* __restrict__ aa, const int64_t* __restrict__ as,
                                   const int32_t* __restrict__ al, const uint8_t* __restrict__ ba,
                                   const int64_t* __restrict__ bs, const int32_t* __restrict__ bl, int64_t n,
                                   int32_t* __restrict__ out, int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* x = aa + as[i];
    const uint8_t* y = ba + bs[i];
    const int32_t lx = al[i], ly = bl[i];
    bool ascii = lx <= kLevMax && ly <= kLevMax;
    for (int32_t k = 0; k < lx && ascii; ++k) ascii = x[k] < 0x80;
    for (int32_t k = 0; k < ly && ascii; ++k) ascii = y[k] < 0x80;
    if (!ascii) { *bad = 1; out[i] = 0; continue; }
    uint16_t row[kLevMax + 1];
    for (int32_t j = 0; j <= ly; ++j) row[j] = (uint16_t)j;
    for (int32_t k = 1; k <= lx; ++k) {
      uint16_t diag = row[0];
      row[0] = (uint16_t)k;
      for (int32_t j = 1; j <= ly; ++j) {
        const uint16_t up = row[j];
        const uint16_t sub = diag + (x[k - 1] != y[j - 1]);
        uint16_t v = up + 1 < row[j - 1] + 1 ? up + 1 : row[j - 1] + 1;
        row[j] = v < sub ? v : sub;
        diag = up;
      }
    }
    out[i] = row[ly];
  }
}

}  // namespace

DXA_API int dxa_pad_args_size() { return (int)sizeof(PadArgs); }

DXA_API int dxa_str_pad(const void* args, const int64_t* off, int64_t* out_len, uint8_t* dst, void* st) {
  const PadArgs& a = *(const PadArgs*)args;
  if (a.n <= 0) return 0;
  if (!off)
    hipLaunchKernelGGL(pad_len_kernel, dim3(dxa_blocks(a.n, 256)), dim3(256), 0, (hipStream_t)st, a, out_len);
  else
    hipLaunchKernelGGL(pad_write_kernel, dim3(dxa_blocks(a.n, 256)), dim3(256), 0, (hipStream_t)st, a, off, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_reverse(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                            const int64_t* off, uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(reverse_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, n,
                     off, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_repeat(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           int64_t times, const int64_t* off, uint8_t* dst, void* st) {
  if (n <= 0 || times <= 0) return 0;
  hipLaunchKernelGGL(repeat_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, n,
                     times, off, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_translate(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                              const uint32_t* from, const int32_t* to, int32_t m, const int64_t* off,
                              int64_t* out_len, uint8_t* dst, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(translate_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, from, to, m, off, out_len, dst);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_initcap(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                            const int64_t* off, uint8_t* dst, int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(initcap_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, n,
                     off, dst, bad);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_substring_index(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                                    const uint8_t* dl, int32_t dn, int64_t count, int64_t* out_start,
                                    int32_t* out_len, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(substring_index_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, n, dl, dn, count, out_start, out_len);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_levenshtein(const uint8_t* aa, const int64_t* as, const int32_t* al, const uint8_t* ba,
                                const int64_t* bs, const int32_t* bl, int64_t n, int32_t* out, int32_t* bad,
                                void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(levenshtein_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, aa, as, al, ba,
                     bs, bl, n, out, bad);
  return (int)hipGetLastError();
}
