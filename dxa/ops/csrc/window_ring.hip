// Dense sliding-window aggregation for gfx950: a persistent group dictionary + a ring of per-pane accumulator rows,
// resident in HBM across micro-batches (SURVEY §2.F K16 "window ring buffer + slicing kernels", the reference's
// past-RDD union + GROUP BY at CommonProcessorFactory.scala:156-236).
//
// A GROUP BY over a 5-minute / 1-second sliding window is answered per batch by
//   1. win_build   — the entering pane's rows look their key hash up in the PERSISTENT open-addressed dictionary
//                    (the table, the slot → group-id map and the group counter survive from batch to batch), new keys
//                    draw the next dense group id; filtered rows (WHERE) go to the dump row ``gcap``;
//   2. win_store   — the first row of each group new to the dictionary copies its key values into fixed-width
//                    dictionary columns (strings up to kKeyWidth bytes), so output keys never point into a pane that
//                    will be evicted;
//   3. win_verify  — every row's key is compared with its dictionary entry (64-bit hash collisions and over-long
//                    strings are reported, never merged: the host then answers the batch the generic way);
//   4. the fused multi-aggregate (hash_groupby.hip agg_multi) accumulates the pane into its ring slot's
//      [group][stride] rows;
//   5. win_combine — the window's ring slots are combined per (group, slot word) in one pass (sum / f64 sum / max —
//                    the accumulator kinds of agg_multi), only for the groups the dictionary holds;
//   6. win_keep    — groups with rows in the window are flagged and counted into the batch's one host read.
// So a batch costs one pane's aggregation plus a (groups × window panes) combine of L2/HBM-resident rows, instead of
// re-grouping ~40 partial tables (the previous paned path), and one synchronising read instead of three.
#include "dxa_common.h"

namespace {

constexpr int kMaxKeyCols = 16;
constexpr int kKeyWidth = 48;            // bytes of a string key kept in the dictionary
enum : int32_t { KC_I64 = 0, KC_F64 = 1, KC_STR = 2 };
enum : int32_t { MA_ADD_U64 = 0, MA_ADD_F64 = 1, MA_MAX_I64 = 2 };

// same layout as hash_groupby.hip's KeyCols (built by dxa/ops/hashing.py key_cols)
struct KeyCol {
  const void* data;
  const int64_t* starts;
  const int32_t* lens;
  const uint8_t* valid;
  int32_t kind;
  int32_t pad;
};
struct KeyCols {
  KeyCol c[kMaxKeyCols];
  int32_t ncols;
  int64_t n;
};

// dictionary key storage, one entry per key column: int64 values (doubles as normalised bit patterns) or
// kKeyWidth-byte string slots + lengths; validity per group
struct DictCol {
  void* vals;          // int64 [gcap + 1]  or  uint8 [(gcap + 1) * kKeyWidth]
  int32_t* lens;       // strings only
  uint8_t* valid;
  int32_t kind;
  int32_t pad;
};
struct DictCols {
  DictCol c[kMaxKeyCols];
  int32_t ncols;
  int32_t gcap;
};

__device__ __forceinline__ uint64_t norm_f64_bits(double d) {
  if (d == 0.0) d = 0.0;                                   // -0.0 groups with 0.0
  uint64_t b = (uint64_t)__double_as_longlong(d);
  return d != d ? 0x7ff8000000000000ull : b;               // one NaN
}

__device__ __forceinline__ uint64_t key_word(const KeyCol& k, int64_t i) {
  return k.kind == KC_F64 ? norm_f64_bits(((const double*)k.data)[i]) : (uint64_t)((const int64_t*)k.data)[i];
}

// 1. dictionary build: persistent table (never re-initialised between batches) → dense group id per row
__global__ void win_build_kernel(const uint64_t* __restrict__ h, const uint8_t* __restrict__ keep, int64_t n,
                                 uint64_t* __restrict__ keys, int64_t cap_mask, int32_t* __restrict__ gid_of_slot,
                                 int32_t* __restrict__ scal, int32_t gcap, int32_t* __restrict__ gid,
                                 int32_t* __restrict__ rep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (keep && !keep[i]) {
      gid[i] = gcap;                                       // filtered row: the dump row, never output
      continue;
    }
    const uint64_t k = dxa::fix_key(h[i]);
    int64_t s = (int64_t)(dxa::fmix64(k) & (uint64_t)cap_mask);
    bool claimed = false;
    int64_t probes = 0;
    while (true) {
      const uint64_t cur = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == k) break;
      if (cur == dxa::kEmpty) {
        const uint64_t prev = atomicCAS((unsigned long long*)&keys[s], (unsigned long long)dxa::kEmpty,
                                        (unsigned long long)k);
        if (prev == dxa::kEmpty) { claimed = true; break; }
        if (prev == k) break;
      }
      s = (s + 1) & cap_mask;
      if (++probes > cap_mask) { s = -1; break; }          // table full (cannot happen while groups < gcap)
    }
    if (s < 0) {
      atomicOr(&scal[1], 2);
      gid[i] = gcap;
      continue;
    }
    int32_t g = -1;
    if (claimed) {
      g = atomicAdd(&scal[0], 1);
      if (g >= gcap) {
        atomicOr(&scal[1], 2);                             // dictionary full: the host falls back
        g = gcap;
      }
      __hip_atomic_store(&gid_of_slot[s], g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!claimed) {
      do {
        g = __hip_atomic_load(&gid_of_slot[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      } while (g < 0);
    }
    gid[i] = g;
    if (g < gcap) atomicMin(&rep[g], (int32_t)i);
  }
}

// 2. the first row (of this batch) of every group whose key is not stored yet writes the dictionary entry
__global__ void win_store_kernel(const KeyCols a, DictCols d, const int32_t* __restrict__ gid,
                                 const int32_t* __restrict__ rep, uint8_t* __restrict__ stored,
                                 int32_t* __restrict__ scal) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = gid[i];
    if (g >= d.gcap || rep[g] != (int32_t)i || stored[g]) continue;
    for (int j = 0; j < a.ncols; ++j) {
      const KeyCol& k = a.c[j];
      const DictCol& e = d.c[j];
      const bool ok = k.valid ? k.valid[i] != 0 : true;
      e.valid[g] = ok ? 1 : 0;
      if (!ok) continue;
      if (k.kind == KC_STR) {
        const int32_t l = k.lens[i];
        if (l > kKeyWidth) {
          atomicOr(&scal[1], 4);                           // key longer than a dictionary slot
          e.lens[g] = 0;
          continue;
        }
        const uint8_t* src = (const uint8_t*)k.data + k.starts[i];
        uint8_t* dst = (uint8_t*)e.vals + (int64_t)g * kKeyWidth;
        for (int32_t q = 0; q < l; ++q) dst[q] = src[q];
        e.lens[g] = l;
      } else {
        ((int64_t*)e.vals)[g] = (int64_t)key_word(k, i);
      }
    }
    stored[g] = 1;
  }
}

// 3. exact check of every row against its dictionary entry
__global__ void win_verify_kernel(const KeyCols a, DictCols d, const int32_t* __restrict__ gid,
                                  int32_t* __restrict__ scal) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = gid[i];
    if (g >= d.gcap) continue;
    bool diff = false;
    for (int j = 0; j < a.ncols && !diff; ++j) {
      const KeyCol& k = a.c[j];
      const DictCol& e = d.c[j];
      const bool vi = k.valid ? k.valid[i] != 0 : true;
      const bool vg = e.valid[g] != 0;
      if (vi != vg) { diff = true; break; }
      if (!vi) continue;
      if (k.kind == KC_STR) {
        const int32_t l = k.lens[i];
        if (l != e.lens[g] || l > kKeyWidth) { diff = true; break; }
        const uint8_t* x = (const uint8_t*)k.data + k.starts[i];
        const uint8_t* y = (const uint8_t*)e.vals + (int64_t)g * kKeyWidth;
        for (int32_t q = 0; q < l && !diff; ++q) diff = x[q] != y[q];
      } else {
        diff = (int64_t)key_word(k, i) != ((const int64_t*)e.vals)[g];
      }
    }
    if (diff) atomicOr(&scal[1], 1);
  }
}

// 5. combine the window's ring slots: out[g][w] = ⊕ over slots s of ring[s][g][w], for g < groups in the dictionary
__global__ __launch_bounds__(256) void win_combine_kernel(const unsigned long long* __restrict__ ring,
                                                          int64_t slot_words, const int32_t* __restrict__ slots,
                                                          int32_t nslots, int32_t stride,
                                                          const int32_t* __restrict__ line_op,
                                                          const int32_t* __restrict__ scal, int32_t gcap,
                                                          int32_t fixed_rows, unsigned long long* __restrict__ out) {
  int32_t ng = fixed_rows > 0 ? fixed_rows : scal[0];
  if (fixed_rows <= 0 && ng > gcap) ng = gcap;
  const int64_t total = (int64_t)ng * stride;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(idx % stride);
    const int op = line_op[w >> 3];
    if (op == MA_ADD_F64) {
      double acc = 0.0;
      for (int s = 0; s < nslots; ++s) acc += __longlong_as_double((long long)ring[(int64_t)slots[s] * slot_words + idx]);
      out[idx] = (unsigned long long)__double_as_longlong(acc);
    } else if (op == MA_ADD_U64) {
      unsigned long long acc = 0;
      for (int s = 0; s < nslots; ++s) acc += ring[(int64_t)slots[s] * slot_words + idx];
      out[idx] = acc;
    } else {
      long long acc = (long long)0x8000000000000000ull;
      for (int s = 0; s < nslots; ++s) {
        const long long v = (long long)ring[(int64_t)slots[s] * slot_words + idx];
        acc = v > acc ? v : acc;
      }
      out[idx] = (unsigned long long)acc;
    }
  }
}

// 6. groups with rows in the window: keep[g] = count word > 0 (count words are f64 sums), counted into scal[2]
__global__ void win_keep_kernel(const unsigned long long* __restrict__ acc, int32_t stride, int32_t count_word,
                                const int32_t* __restrict__ scal_in, int32_t gcap, uint8_t* __restrict__ keep,
                                int32_t* __restrict__ scal) {
  int32_t ng = scal_in[0];
  if (ng > gcap) ng = gcap;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < gcap; g += (int64_t)gridDim.x * blockDim.x) {
    bool k = false;
    if (g < ng) k = __longlong_as_double((long long)acc[g * stride + count_word]) > 0.0;
    keep[g] = k ? 1 : 0;
    if (k) atomicAdd(&scal[2], 1);
  }
}

// exclusive positions of the kept groups (one block-sequential scan is enough for ≤ 2^20 groups: the keep flags
// are scanned by a single workgroup in 256-wide chunks) → out_idx[pos] = g
__global__ __launch_bounds__(256) void win_compact_kernel(const uint8_t* __restrict__ keep, int32_t gcap,
                                                          const int32_t* __restrict__ scal,
                                                          int64_t* __restrict__ out_idx) {
  __shared__ int32_t part[256];
  int32_t base = 0;
  int32_t ng = scal[0];
  if (ng > gcap) ng = gcap;
  for (int32_t c0 = 0; c0 < ng; c0 += 256 * 16) {
    // each thread counts 16 consecutive flags
    const int32_t lo = c0 + threadIdx.x * 16;
    int32_t cnt = 0;
    for (int q = 0; q < 16; ++q) cnt += (lo + q < ng && keep[lo + q]) ? 1 : 0;
    part[threadIdx.x] = cnt;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {              // inclusive scan of the 256 counts
      const int32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += v;
      __syncthreads();
    }
    int32_t pos = base + part[threadIdx.x] - cnt;
    for (int q = 0; q < 16; ++q) {
      const int32_t g = lo + q;
      if (g < ng && keep[g]) out_idx[pos++] = g;
    }
    base += part[255];
    __syncthreads();
  }
}

__global__ void win_fill_i32_kernel(int32_t* __restrict__ p, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

}  // namespace

DXA_API int dxa_win_sizes(int32_t* out) {
  out[0] = (int32_t)sizeof(KeyCols);
  out[1] = (int32_t)sizeof(DictCols);
  out[2] = kKeyWidth;
  return 0;
}

// table init (once per dictionary): keys = empty, gid_of_slot = -1
DXA_API int dxa_win_init(uint64_t* keys, int32_t* gid_of_slot, int64_t cap, void* st) {
  hipStream_t s = (hipStream_t)st;
  hipMemsetAsync(keys, 0xFF, (size_t)cap * 8, s);
  hipMemsetAsync(gid_of_slot, 0xFF, (size_t)cap * 4, s);
  return (int)hipGetLastError();
}

// steps 1-3 for one pane: h [n], keep [n] or null; rep [gcap] scratch (re-filled here); scal = {groups, bad, kept}
DXA_API int dxa_win_insert(const uint64_t* h, const uint8_t* keep, int64_t n, uint64_t* keys, int64_t cap,
                           int32_t* gid_of_slot, int32_t* scal, int32_t gcap, int32_t* gid, int32_t* rep,
                           const void* keycols, const void* dictcols, uint8_t* stored, void* st) {
  hipStream_t s = (hipStream_t)st;
  hipLaunchKernelGGL(win_fill_i32_kernel, dim3(dxa_blocks(gcap, 256)), dim3(256), 0, s, rep, (int64_t)gcap,
                     (int32_t)0x7fffffff);
  if (n <= 0) return (int)hipGetLastError();
  const int blocks = dxa_blocks(n, 256);
  hipLaunchKernelGGL(win_build_kernel, dim3(blocks), dim3(256), 0, s, h, keep, n, keys, cap - 1, gid_of_slot, scal,
                     gcap, gid, rep);
  const KeyCols& a = *(const KeyCols*)keycols;
  const DictCols& d = *(const DictCols*)dictcols;
  hipLaunchKernelGGL(win_store_kernel, dim3(blocks), dim3(256), 0, s, a, d, gid, rep, stored, scal);
  hipLaunchKernelGGL(win_verify_kernel, dim3(blocks), dim3(256), 0, s, a, d, gid, scal);
  return (int)hipGetLastError();
}

// steps 5-6 + compaction: ring [R][(gcap+1)*stride] u64, slots [nslots] (device), out acc [(gcap+1)*stride],
// keep [gcap] scratch, out_idx [gcap] (the first scal[2] entries are the kept groups, in group order)
DXA_API int dxa_win_combine(const void* ring, int32_t gcap, int32_t stride, const int32_t* slots, int32_t nslots,
                            const int32_t* line_op, int32_t count_word, int32_t* scal, void* acc, uint8_t* keep,
                            int64_t* out_idx, void* st) {
  hipStream_t s = (hipStream_t)st;
  const int64_t slot_words = (int64_t)(gcap + 1) * stride;
  hipMemsetAsync(scal + 2, 0, 4, s);
  hipLaunchKernelGGL(win_combine_kernel, dim3(dxa_blocks((int64_t)gcap * stride, 256, 256 * 64)), dim3(256), 0, s,
                     (const unsigned long long*)ring, slot_words, slots, nslots, stride, line_op, scal, gcap, 0,
                     (unsigned long long*)acc);
  hipLaunchKernelGGL(win_keep_kernel, dim3(dxa_blocks(gcap, 256)), dim3(256), 0, s,
                     (const unsigned long long*)acc, stride, count_word, scal, gcap, keep, scal);
  hipLaunchKernelGGL(win_compact_kernel, dim3(1), dim3(256), 0, s, keep, gcap, scal, out_idx);
  return (int)hipGetLastError();
}

// a block of ring slots pre-combined into another ring slot (every row, so groups the dictionary gains later read
// the identity there): out = ring slot ``dst``
DXA_API int dxa_win_combine_block(void* ring, int32_t gcap, int32_t stride, const int32_t* slots, int32_t nslots,
                                  const int32_t* line_op, int32_t dst, void* st) {
  hipStream_t s = (hipStream_t)st;
  const int64_t slot_words = (int64_t)(gcap + 1) * stride;
  unsigned long long* r = (unsigned long long*)ring;
  hipLaunchKernelGGL(win_combine_kernel, dim3(dxa_blocks((int64_t)(gcap + 1) * stride, 256, 256 * 64)), dim3(256), 0,
                     s, (const unsigned long long*)r, slot_words, slots, nslots, stride, line_op, (const int32_t*)nullptr,
                     gcap, gcap + 1, r + (int64_t)dst * slot_words);
  return (int)hipGetLastError();
}
