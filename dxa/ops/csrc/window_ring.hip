// Dense sliding-window aggregation for gfx950: a persistent group dictionary + a ring of per-pane accumulator rows,
// resident in HBM across micro-batches (SURVEY §2.F K16 "window ring buffer + slicing kernels", the reference's
// past-RDD union + GROUP BY at CommonProcessorFactory.scala:156-236).
//
// A GROUP BY over a 5-minute / 1-second sliding window is answered per batch by
//   1. win_insert  — the entering pane's rows hash their key and look it up in the PERSISTENT open-addressed
//                    dictionary (the table, the slot → group-id map and the group counter survive from batch to
//                    batch); a new key draws the next dense group id and its claiming lane copies the key values into
//                    fixed-width dictionary columns (strings up to kKeyWidth bytes) before publishing the id, so
//                    output keys never point into a pane that will be evicted; every other row compares its key with
//                    the entry (64-bit hash collisions and over-long strings are reported, never merged: the host then
//                    answers the batch the generic way); filtered rows (WHERE) go to the dump row ``gcap``;
//   2. the fused multi-aggregate (hash_groupby.hip agg_multi) accumulates the pane into its ring slot's
//      [group][stride] rows (complete blocks of panes are pre-combined into block slots once);
//   3. win_combine — the window's ring / block slots are combined per (group, word) in one pass (sum / f64 sum / max
//                    — the accumulator kinds of agg_multi), only for the groups the dictionary holds;
//   4. win_keep + win_compact — groups with rows in the window are flagged, counted into the batch's one host read
//                    and listed in group order;
//   5. win_emit    — every kept group's key columns and finished aggregates are written by output position, so the
//                    host only slices the outputs after its read.
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



__device__ __forceinline__ uint64_t row_hash(const KeyCols& a, int64_t i) {
  uint64_t h = 0;
  for (int j = 0; j < a.ncols; ++j) {
    const KeyCol& k = a.c[j];
    uint64_t x;
    if (k.valid && !k.valid[i]) x = dxa::kNullHash;
    else if (k.kind == KC_STR) x = dxa::hash_bytes((const uint8_t*)k.data + k.starts[i], k.lens[i]);
    else x = dxa::hash_i64(key_word(k, i));
    h = j ? dxa::hash_combine(h, x) : x;
  }
  return h;
}

// store row i's key as group g's dictionary entry (the claiming lane, before it publishes g)
__device__ __forceinline__ void store_key(const KeyCols& a, const DictCols& d, int64_t i, int32_t g,
                                          int32_t* __restrict__ scal) {
  for (int j = 0; j < a.ncols; ++j) {
    const KeyCol& k = a.c[j];
    const DictCol& e = d.c[j];
    const bool ok = k.valid ? k.valid[i] != 0 : true;
    e.valid[g] = ok ? 1 : 0;
    if (!ok) continue;
    if (k.kind == KC_STR) {
      const int32_t l = k.lens[i];
      if (l > kKeyWidth) {
        atomicOr(&scal[1], 4);
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
}

__device__ __forceinline__ bool key_differs(const KeyCols& a, const DictCols& d, int64_t i, int32_t g) {
  for (int j = 0; j < a.ncols; ++j) {
    const KeyCol& k = a.c[j];
    const DictCol& e = d.c[j];
    const bool vi = k.valid ? k.valid[i] != 0 : true;
    if (vi != (e.valid[g] != 0)) return true;
    if (!vi) continue;
    if (k.kind == KC_STR) {
      const int32_t l = k.lens[i];
      if (l != e.lens[g] || l > kKeyWidth) return true;
      // 8 bytes per step (dxa::load_le): the slot is 8-byte aligned, the row's bytes are not
      const uint8_t* x = (const uint8_t*)k.data + k.starts[i];
      const uint64_t* y = (const uint64_t*)((const uint8_t*)e.vals + (int64_t)g * kKeyWidth);
      for (int32_t q = 0; q < l; q += 8) {
        const int32_t nb = l - q < 8 ? l - q : 8;
        const uint64_t yw = nb < 8 ? y[q >> 3] & ((1ull << (8 * nb)) - 1ull) : y[q >> 3];
        if (dxa::load_le(x + q, nb) != yw) return true;
      }
    } else if ((int64_t)key_word(k, i) != ((const int64_t*)e.vals)[g]) {
      return true;
    }
  }
  return false;
}

// steps 1-3 in ONE pass: hash the row's key, look it up in the persistent dictionary; the lane whose CAS claims a
// new entry draws the group id, writes the key into the dictionary and only then publishes the id (release), so a
// lane that finds the entry (acquire) compares its key with a complete dictionary entry — a 64-bit collision or a
// key too long for a slot is flagged, never merged.  Claims and publications precede every wait in straight-line
// code (as hash_groupby.hip group_build_kernel): a waiting lane only waits on another wave.
__global__ void win_insert_kernel(const KeyCols a, DictCols d, const uint8_t* __restrict__ keep,
                                  uint64_t* __restrict__ keys, int64_t cap_mask,
                                  int32_t* __restrict__ gid_of_slot, int32_t* __restrict__ scal,
                                  int32_t* __restrict__ gid) {
  const int32_t gcap = d.gcap;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    if (keep && !keep[i]) {
      gid[i] = gcap;
      continue;
    }
    const uint64_t k = dxa::fix_key(row_hash(a, i));
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
      if (++probes > cap_mask) { s = -1; break; }
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
        atomicOr(&scal[1], 2);
        g = gcap;
      } else {
        store_key(a, d, i, g, scal);
      }
      __hip_atomic_store(&gid_of_slot[s], g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!claimed) {
      do {
        g = __hip_atomic_load(&gid_of_slot[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      } while (g < 0);
      if (g < gcap && key_differs(a, d, i, g)) atomicOr(&scal[1], 1);
    }
    gid[i] = g;
  }
}

// The window's output rows, written once by position (no gather launches afterwards): position p < kept holds
// group out_idx[p]: its key columns (int64 words / the string's dictionary slot) and every requested aggregate
// finished from the combined accumulator row (the kinds of hash_groupby.hip agg_finish_kernel).  Outputs are
// [gcap]-strided; the host slices the first ``kept`` entries after its one read.
constexpr int kMaxEmit = 64;
enum : int { F_COUNT = 0, F_I64 = 1, F_F64 = 2, F_AVG = 3, F_F64_ORD = 4, F_NOT = 8 };
struct EmitArgs {
  const long long* acc;
  int32_t stride;
  int32_t nreq;
  int32_t kind[kMaxEmit];
  int32_t pos[kMaxEmit];
  int32_t cnt[kMaxEmit];
  long long* dst;                // [nreq][gcap]
  uint8_t* dvalid;               // [nreq][gcap]
  int64_t* okey[kMaxKeyCols];    // [gcap] int64 key words, or the strings' starts in the dictionary arena
  int32_t* olen[kMaxKeyCols];    // strings: [gcap] lengths
  uint8_t* ovalid[kMaxKeyCols];  // [gcap]
  const int64_t* out_idx;
  const int32_t* scal;
  int32_t gcap;
};

__global__ __launch_bounds__(256) void win_emit_kernel(const EmitArgs e, DictCols d) {
  const int32_t kept = e.scal[2];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < kept; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = e.out_idx[p];
    for (int j = 0; j < d.ncols; ++j) {
      const DictCol& c = d.c[j];
      e.ovalid[j][p] = c.valid[g];
      if (c.kind == KC_STR) {
        e.okey[j][p] = g * kKeyWidth;
        e.olen[j][p] = c.lens[g];
      } else {
        e.okey[j][p] = ((const int64_t*)c.vals)[g];
      }
    }
    const long long* row = e.acc + g * e.stride;
    for (int r = 0; r < e.nreq; ++r) {
      const int k = e.kind[r];
      long long v = row[e.pos[r]];
      if (k & F_NOT) v = ~v;
      const double c = e.cnt[r] >= 0 ? __longlong_as_double(row[e.cnt[r]]) : 1.0;
      long long o;
      switch (k & 7) {
        case F_COUNT: o = (long long)__longlong_as_double(v); break;
        case F_AVG: o = __double_as_longlong(__longlong_as_double(v) / (c > 1.0 ? c : 1.0)); break;
        case F_F64_ORD: o = v < 0 ? (v ^ 0x7fffffffffffffffll) : v; break;
        default: o = v; break;
      }
      e.dst[(int64_t)r * e.gcap + p] = o;
      e.dvalid[(int64_t)r * e.gcap + p] = c > 0.0 ? 1 : 0;
    }
  }
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

DXA_API int dxa_win_emit_size() { return (int)sizeof(EmitArgs); }

// one pane into the dictionary (fused hash + lookup / claim + key store + verify)
DXA_API int dxa_win_insert_fused(const void* keycols, const void* dictcols, const uint8_t* keep, uint64_t* keys,
                                 int64_t cap, int32_t* gid_of_slot, int32_t* scal, int32_t* gid, void* st) {
  const KeyCols& a = *(const KeyCols*)keycols;
  if (a.n <= 0) return 0;
  hipLaunchKernelGGL(win_insert_kernel, dim3(dxa_blocks(a.n, 256)), dim3(256), 0, (hipStream_t)st, a,
                     *(const DictCols*)dictcols, keep, keys, cap - 1, gid_of_slot, scal, gid);
  return (int)hipGetLastError();
}

// steps 5-6, compaction and the output rows by position (win_emit_kernel)
DXA_API int dxa_win_answer(const void* ring, int32_t gcap, int32_t stride, const int32_t* slots, int32_t nslots,
                           const int32_t* line_op, int32_t count_word, int32_t* scal, void* acc, uint8_t* keep,
                           int64_t* out_idx, const void* emit, const void* dictcols, void* st) {
  const int rc = dxa_win_combine(ring, gcap, stride, slots, nslots, line_op, count_word, scal, acc, keep, out_idx,
                                 st);
  if (rc) return rc;
  hipLaunchKernelGGL(win_emit_kernel, dim3(dxa_blocks(gcap, 256)), dim3(256), 0, (hipStream_t)st,
                     *(const EmitArgs*)emit, *(const DictCols*)dictcols);
  return (int)hipGetLastError();
}
