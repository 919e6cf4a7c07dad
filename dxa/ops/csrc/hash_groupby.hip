// Hashing, hash group-by / aggregation and hash-join kernels for gfx950 (kernels K11, K12, K13 in SURVEY §2.F).
//
// Group-by is three launches, none of which spins on another lane (a spin inside one wave64 can deadlock when
// the publishing lane sits in the same wave):
//   1. insert   — each row CASes its 64-bit key hash into an open-addressed table (capacity ≥ 2×rows, linear
//                 probing) and records the slot it landed in;
//   2. number   — every occupied slot draws a dense group id (one atomic per group, not per row);
//   3. gather   — row → group id, and representative row = min row index of the group (atomicMin).
// Aggregation then privatises per-group accumulators in LDS when the group count is small (the IoT flows have
// 10^1–10^4 groups against 10^6+ rows — global atomics on a handful of hot lines would serialise on the memory
// side, MI355X_MICROARCH.md "Global float atomics": one row hammered = 14× slower), and flushes one global atomic
// per (workgroup, group).  Large group counts go straight to global atomics, which then rarely contend.
//
// Join: build side rows are inserted the same way (slot per build row), bucketed by counting sort over slots, and
// probed with a count pass + exclusive scan + write pass.  Exact key equality is re-checked afterwards on the
// host-visible columns (hash collisions are filtered, never silently merged).
#include "dxa_common.h"

namespace {

using dxa::fmix64;

// ------------------------------------------------------------------------------------------------------------
// hashing
// ------------------------------------------------------------------------------------------------------------
__global__ void hash_i64_kernel(const int64_t* __restrict__ v, const uint8_t* __restrict__ valid, int64_t n,
                                uint64_t* __restrict__ out, int combine) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = (valid && !valid[i]) ? dxa::kNullHash : dxa::hash_i64((uint64_t)v[i]);
    out[i] = combine ? dxa::hash_combine(out[i], h) : h;
  }
}

__global__ void hash_f64_kernel(const double* __restrict__ v, const uint8_t* __restrict__ valid, int64_t n,
                                uint64_t* __restrict__ out, int combine) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h;
    if (valid && !valid[i]) {
      h = dxa::kNullHash;
    } else {
      double d = v[i];
      if (d == 0.0) d = 0.0;                       // -0.0 → 0.0
      uint64_t bits = (uint64_t)__double_as_longlong(d);
      if (d != d) bits = 0x7ff8000000000000ull;   // canonical NaN
      h = dxa::hash_i64(bits);
    }
    out[i] = combine ? dxa::hash_combine(out[i], h) : h;
  }
}

__global__ void hash_str_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                                uint64_t* __restrict__ out, int combine) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = (valid && !valid[i]) ? dxa::kNullHash : dxa::hash_bytes(arena + starts[i], lens[i]);
    out[i] = combine ? dxa::hash_combine(out[i], h) : h;
  }
}

// Several key columns in ONE launch: the per-column hashes above, combined in column order exactly as the
// one-launch-per-column sequence combines them (so both paths give the same bits), and the matching equality check
// against each row's group representative.
constexpr int kMaxKeyCols = 16;
enum : int32_t { KC_I64 = 0, KC_F64 = 1, KC_STR = 2 };

struct KeyCol {
  const void* data;        // int64 / double values, or the string arena
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

__device__ __forceinline__ uint64_t key_hash(const KeyCol& k, int64_t i) {
  if (k.valid && !k.valid[i]) return dxa::kNullHash;
  if (k.kind == KC_STR) return dxa::hash_bytes((const uint8_t*)k.data + k.starts[i], k.lens[i]);
  if (k.kind == KC_F64) {
    double d = ((const double*)k.data)[i];
    if (d == 0.0) d = 0.0;
    uint64_t bits = (uint64_t)__double_as_longlong(d);
    if (d != d) bits = 0x7ff8000000000000ull;
    return dxa::hash_i64(bits);
  }
  return dxa::hash_i64((uint64_t)((const int64_t*)k.data)[i]);
}

__global__ void hash_multi_kernel(const KeyCols a, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = key_hash(a.c[0], i);
    for (int j = 1; j < a.ncols; ++j) h = dxa::hash_combine(h, key_hash(a.c[j], i));
    out[i] = h;
  }
}

__device__ __forceinline__ uint64_t load_part(const uint8_t* p, int32_t avail);

__global__ void verify_multi_kernel(const KeyCols a, const int32_t* __restrict__ gid, const int32_t* __restrict__ rep,
                                    int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = rep[gid[i]];
    bool diff = false;
    for (int j = 0; j < a.ncols && !diff; ++j) {
      const KeyCol& k = a.c[j];
      const bool vi = k.valid ? k.valid[i] != 0 : true;
      const bool vr = k.valid ? k.valid[r] != 0 : true;
      diff = vi != vr;
      if (diff || !vi) continue;
      if (k.kind == KC_STR) {
        const int32_t l = k.lens[i];
        if (l != k.lens[r]) { diff = true; continue; }
        const uint8_t* x = (const uint8_t*)k.data + k.starts[i];
        const uint8_t* y = (const uint8_t*)k.data + k.starts[r];
        for (int32_t q = 0; q < l && !diff; q += 8) {
          const int32_t av = l - q < 8 ? l - q : 8;
          diff = load_part(x + q, av) != load_part(y + q, av);
        }
      } else {
        diff = ((const int64_t*)k.data)[i] != ((const int64_t*)k.data)[r];     // bit equality (as verify_i64)
      }
    }
    if (diff) atomicAdd(bad, 1);
  }
}

// Join candidate pairs: out[j] = (ri[j] >= 0) and every key column of left row li[j] equals right row ri[j] (SQL
// equality: a NULL on either side never matches; doubles compare as numbers).  One launch for all key columns.
__global__ void pairs_equal_kernel(const KeyCols L, const KeyCols R, const int64_t* __restrict__ li,
                                   const int64_t* __restrict__ ri, int64_t m, uint8_t* __restrict__ out) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = li[j], b = ri[j];
    bool eq = b >= 0;
    for (int c = 0; c < L.ncols && eq; ++c) {
      const KeyCol& x = L.c[c];
      const KeyCol& y = R.c[c];
      if ((x.valid && !x.valid[a]) || (y.valid && !y.valid[b])) { eq = false; break; }
      if (x.kind == KC_STR) {
        const int32_t l = x.lens[a];
        if (l != y.lens[b]) { eq = false; break; }
        const uint8_t* p = (const uint8_t*)x.data + x.starts[a];
        const uint8_t* q = (const uint8_t*)y.data + y.starts[b];
        for (int32_t k = 0; k < l && eq; k += 8) {
          const int32_t av = l - k < 8 ? l - k : 8;
          eq = load_part(p + k, av) == load_part(q + k, av);
        }
      } else if (x.kind == KC_F64) {
        eq = ((const double*)x.data)[a] == ((const double*)y.data)[b];
      } else {
        eq = ((const int64_t*)x.data)[a] == ((const int64_t*)y.data)[b];
      }
    }
    out[j] = eq ? 1 : 0;
  }
}

// ------------------------------------------------------------------------------------------------------------
// group-by: insert / number / gather
// ------------------------------------------------------------------------------------------------------------
__global__ void table_insert_kernel(const uint64_t* __restrict__ h, int64_t n, uint64_t* __restrict__ keys,
                                    int64_t cap_mask, int32_t* __restrict__ slot_of_row) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = dxa::fix_key(h[i]);
    int64_t s = (int64_t)(fmix64(k) & (uint64_t)cap_mask);
    while (true) {
      const uint64_t cur = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == k) break;
      if (cur == dxa::kEmpty) {
        const uint64_t prev = atomicCAS((unsigned long long*)&keys[s], (unsigned long long)dxa::kEmpty,
                                        (unsigned long long)k);
        if (prev == dxa::kEmpty || prev == k) break;
      }
      s = (s + 1) & cap_mask;
    }
    slot_of_row[i] = (int32_t)s;
  }
}

// Insert + number + gather in ONE pass: the lane whose CAS claims an empty slot takes the next group id from a
// counter and publishes it in gid_of_slot (pre-filled with -1); lanes that find the key already present wait for
// that id.  The claim and the publication come before any lane of the wave waits (straight-line code, then a
// reconvergent spin), so a waiting lane only ever waits on another wave.  Ids come out in claim order; the host
// renumbers them by first row (dxa_group_renumber).  Replaces the table_number scan over every slot of the table.
__global__ void group_build_kernel(const uint64_t* __restrict__ h, int64_t n, uint64_t* __restrict__ keys,
                                   int64_t cap_mask, int32_t* __restrict__ gid_of_slot, int32_t* __restrict__ counter,
                                   int32_t* __restrict__ gid, int32_t* __restrict__ rep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = dxa::fix_key(h[i]);
    int64_t s = (int64_t)(fmix64(k) & (uint64_t)cap_mask);
    bool claimed = false;
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
    }
    int32_t g = -1;
    if (claimed) {
      g = atomicAdd(counter, 1);
      __hip_atomic_store(&gid_of_slot[s], g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!claimed) {
      do {
        g = __hip_atomic_load(&gid_of_slot[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      } while (g < 0);
    }
    gid[i] = g;
    atomicMin(&rep[g], (int32_t)i);
  }
}

__global__ void table_number_kernel(const uint64_t* __restrict__ keys, int64_t cap, int32_t* __restrict__ gid_of_slot,
                                    int32_t* __restrict__ counter) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += (int64_t)gridDim.x * blockDim.x) {
    gid_of_slot[s] = keys[s] != dxa::kEmpty ? atomicAdd(counter, 1) : -1;
  }
}

__global__ void group_gather_kernel(const int32_t* __restrict__ slot_of_row, const int32_t* __restrict__ gid_of_slot,
                                    int64_t n, int32_t* __restrict__ gid, int32_t* __restrict__ rep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t g = gid_of_slot[slot_of_row[i]];
    gid[i] = g;
    atomicMin(&rep[g], (int32_t)i);
  }
}

// Exact-key verification: flag rows whose key columns differ from their group representative's.
__global__ void verify_i64_kernel(const int64_t* __restrict__ v, const uint8_t* __restrict__ valid,
                                  const int32_t* __restrict__ gid, const int32_t* __restrict__ rep, int64_t n,
                                  int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = rep[gid[i]];
    const bool vi = valid ? valid[i] != 0 : true;
    const bool vr = valid ? valid[r] != 0 : true;
    if (vi != vr || (vi && v[i] != v[r])) atomicAdd(bad, 1);
  }
}

// bytes [p, p + avail) (avail <= 8) as one little-endian word, read from the aligned words that overlap them only
__device__ __forceinline__ uint64_t load_part(const uint8_t* p, int32_t avail) {
  const uintptr_t x = reinterpret_cast<uintptr_t>(p);
  const int m = (int)(x & 7);
  const uint64_t* q = reinterpret_cast<const uint64_t*>(x - m);
  uint64_t v = q[0] >> (8 * m);
  if (m && 8 - m < avail) v |= q[1] << (64 - 8 * m);
  if (avail < 8) v &= (1ull << (8 * avail)) - 1;
  return v;
}

__global__ void verify_str_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid,
                                  const int32_t* __restrict__ gid, const int32_t* __restrict__ rep, int64_t n,
                                  int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = rep[gid[i]];
    const bool vi = valid ? valid[i] != 0 : true;
    const bool vr = valid ? valid[r] != 0 : true;
    bool diff = vi != vr;
    if (!diff && vi) {
      const int32_t l = lens[i];
      if (l != lens[r]) diff = true;
      else {
        const uint8_t* a = arena + starts[i];
        const uint8_t* b = arena + starts[r];
        for (int32_t k = 0; k < l && !diff; k += 8) {
          const int32_t av = l - k < 8 ? l - k : 8;
          diff = load_part(a + k, av) != load_part(b + k, av);
        }
      }
    }
    if (diff) atomicAdd(bad, 1);
  }
}

// ------------------------------------------------------------------------------------------------------------
// aggregation
// ------------------------------------------------------------------------------------------------------------
enum : int32_t { AGG_SUM = 0, AGG_MIN = 1, AGG_MAX = 2, AGG_COUNT = 3 };
enum : int32_t { VT_I64 = 0, VT_F64 = 1 };

__device__ __forceinline__ void lds_f64_min(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a, assumed;
  do {
    assumed = old;
    if (__longlong_as_double((long long)assumed) <= v) return;
    old = atomicCAS(a, assumed, (unsigned long long)__double_as_longlong(v));
  } while (old != assumed);
}
__device__ __forceinline__ void lds_f64_max(double* p, double v) {
  unsigned long long* a = (unsigned long long*)p;
  unsigned long long old = *a, assumed;
  do {
    assumed = old;
    if (__longlong_as_double((long long)assumed) >= v) return;
    old = atomicCAS(a, assumed, (unsigned long long)__double_as_longlong(v));
  } while (old != assumed);
}

template <int VT, int OP>
__device__ __forceinline__ void acc_update(void* accp, int32_t g, const void* vals, int64_t i) {
  if constexpr (OP == AGG_COUNT) {
    atomicAdd(((unsigned long long*)accp) + g, 1ull);
  } else if constexpr (VT == VT_I64) {
    long long* acc = (long long*)accp;
    const long long v = ((const long long*)vals)[i];
    if constexpr (OP == AGG_SUM) atomicAdd((unsigned long long*)&acc[g], (unsigned long long)v);
    else if constexpr (OP == AGG_MIN) atomicMin(&acc[g], v);
    else atomicMax(&acc[g], v);
  } else {
    double* acc = (double*)accp;
    const double v = ((const double*)vals)[i];
    if constexpr (OP == AGG_SUM) atomicAdd(&acc[g], v);
    else if constexpr (OP == AGG_MIN) lds_f64_min(&acc[g], v);
    else lds_f64_max(&acc[g], v);
  }
}

template <int VT, int OP>
__device__ __forceinline__ uint64_t identity_bits() {
  if constexpr (OP == AGG_SUM || OP == AGG_COUNT) return 0ull;
  if constexpr (VT == VT_I64) return OP == AGG_MIN ? 0x7fffffffffffffffull : 0x8000000000000000ull;
  return OP == AGG_MIN ? 0x7ff0000000000000ull /* +inf */ : 0xfff0000000000000ull /* -inf */;
}

// LDS-privatised aggregation: one accumulator array of ngroups per workgroup.
template <int VT, int OP>
__global__ __launch_bounds__(256) void agg_lds_kernel(const int32_t* __restrict__ gid, const void* __restrict__ vals,
                                                      const uint8_t* __restrict__ valid, int64_t n, int32_t ngroups,
                                                      void* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_acc[];
  for (int g = threadIdx.x; g < ngroups; g += blockDim.x) lds_acc[g] = identity_bits<VT, OP>();
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) continue;
    acc_update<VT, OP>((void*)lds_acc, gid[i], vals, i);
  }
  __syncthreads();
  for (int g = threadIdx.x; g < ngroups; g += blockDim.x) {
    const unsigned long long b = lds_acc[g];
    if (b == identity_bits<VT, OP>() && OP != AGG_SUM) continue;
    if constexpr (OP == AGG_COUNT) {
      if (b) atomicAdd(((unsigned long long*)out) + g, b);
    } else if constexpr (VT == VT_I64) {
      long long* o = (long long*)out;
      if constexpr (OP == AGG_SUM) { if (b) atomicAdd((unsigned long long*)&o[g], b); }
      else if constexpr (OP == AGG_MIN) atomicMin(&o[g], (long long)b);
      else atomicMax(&o[g], (long long)b);
    } else {
      double* o = (double*)out;
      const double v = __longlong_as_double((long long)b);
      if constexpr (OP == AGG_SUM) { if (b) atomicAdd(&o[g], v); }
      else if constexpr (OP == AGG_MIN) lds_f64_min(&o[g], v);
      else lds_f64_max(&o[g], v);
    }
  }
}

template <int VT, int OP>
__global__ __launch_bounds__(256) void agg_global_kernel(const int32_t* __restrict__ gid, const void* __restrict__ vals,
                                                         const uint8_t* __restrict__ valid, int64_t n,
                                                         void* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) continue;
    acc_update<VT, OP>(out, gid[i], vals, i);
  }
}

template <int VT, int OP>
__global__ void agg_init_kernel(void* out, int32_t ngroups) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ngroups) ((unsigned long long*)out)[g] = identity_bits<VT, OP>();
}

template <int VT, int OP>
int launch_agg(const int32_t* gid, const void* vals, const uint8_t* valid, int64_t n, int32_t ngroups, void* out,
               hipStream_t s) {
  hipLaunchKernelGGL((agg_init_kernel<VT, OP>), dim3((ngroups + 255) / 256), dim3(256), 0, s, out, ngroups);
  if (n <= 0) return (int)hipGetLastError();
  const size_t lds = (size_t)ngroups * 8;
  if (ngroups <= 8192) {
    // ≈ 2 blocks per CU of streaming work; each block then flushes ngroups atomics.
    int blocks = dxa_blocks(n, 256, ngroups <= 1024 ? 1024 : 512);
    hipLaunchKernelGGL((agg_lds_kernel<VT, OP>), dim3(blocks), dim3(256), lds, s, gid, vals, valid, n, ngroups, out);
  } else {
    hipLaunchKernelGGL((agg_global_kernel<VT, OP>), dim3(dxa_blocks(n, 256, 4096)), dim3(256), 0, s, gid, vals,
                       valid, n, out);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------------------
// fused multi-aggregate (many groups).  Global atomics execute at the memory side, one 64-B request per distinct
// line touched by a wave instruction (MI355X_MICROARCH.md "Global float atomics"), so the cost of a group-by with
// 10^4 groups is the request count, not the bytes.  All of a query's simple aggregates therefore live in one
// [group][stride] u64 row, slots of one atomic kind packed into the same 8-slot (64-B) line; eight lanes serve one
// input row, lane j updating slot 8L+j of line L.  One wave instruction then touches one line per row for up to
// eight aggregates.  MIN is folded into MAX (of the bitwise complement) and counts are f64 adds (exact below 2^53),
// so the IoT GROUP BY's 12 per-row atomics become 2 requests.
// ------------------------------------------------------------------------------------------------------------
enum : int32_t { MA_ADD_U64 = 0, MA_ADD_F64 = 1, MA_MAX_I64 = 2 };
enum : int32_t { MV_SKIP = -1, MV_COUNT = 0, MV_I64 = 1, MV_F64 = 2, MV_F64_ORD = 3, MV_NOT = 4 };
constexpr int kMaxAggSlots = 64;

struct MultiAggSlot {
  const void* data;
  const uint8_t* valid;
  int64_t kind;
};

struct MultiAggArgs {
  const int32_t* gid;
  int64_t n;
  int32_t nslots;
  int32_t nlines;
  int32_t line_op[kMaxAggSlots / 8];
  unsigned long long* out;
  MultiAggSlot slot[kMaxAggSlots];
};

// total order of doubles as signed 64-bit integers (NaN canonical and greatest, as Spark orders it)
__device__ __forceinline__ long long f64_ordered(double d) {
  long long b = __double_as_longlong(d);
  if (d != d) b = 0x7ff8000000000000ll;
  return b >= 0 ? b : (b ^ 0x7fffffffffffffffll);
}

__global__ __launch_bounds__(256) void agg_multi_init_kernel(MultiAggArgs a, int32_t ngroups) {
  const int64_t total = (int64_t)ngroups * a.nlines * 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int op = a.line_op[(int)((i / 8) % a.nlines)];
    a.out[i] = op == MA_MAX_I64 ? 0x8000000000000000ull : 0ull;
  }
}

__global__ __launch_bounds__(256) void agg_multi_kernel(MultiAggArgs a) {
  __shared__ MultiAggSlot sl[kMaxAggSlots];
  for (int i = threadIdx.x; i < a.nslots; i += blockDim.x) sl[i] = a.slot[i];
  __syncthreads();
  const int j = threadIdx.x & 7;
  const int stride = a.nlines * 8;
  const int64_t step = ((int64_t)gridDim.x * blockDim.x) >> 3;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3; r < a.n; r += step) {
    unsigned long long* row = a.out + (int64_t)a.gid[r] * stride;
    for (int L = 0; L < a.nlines; ++L) {
      const int s = L * 8 + j;
      if (s >= a.nslots) continue;
      const MultiAggSlot d = sl[s];
      if (d.kind == MV_SKIP || (d.valid && !d.valid[r])) continue;
      const int op = a.line_op[L];
      const int kind = (int)(d.kind & 3);
      if (op == MA_ADD_F64) {
        const double v = kind == MV_COUNT ? 1.0 : static_cast<const double*>(d.data)[r];
        atomicAdd(reinterpret_cast<double*>(row + s), v);
      } else if (op == MA_ADD_U64) {
        atomicAdd(row + s, kind == MV_COUNT ? 1ull : static_cast<const unsigned long long*>(d.data)[r]);
      } else {
        long long v = kind == MV_F64_ORD ? f64_ordered(static_cast<const double*>(d.data)[r])
                                         : static_cast<const long long*>(d.data)[r];
        if (d.kind & MV_NOT) v = ~v;                   // MIN(x) = ~MAX(~x): one atomic kind, one line
        atomicMax(reinterpret_cast<long long*>(row + s), v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// hash join (build = slot buckets, probe = count + write)
// ------------------------------------------------------------------------------------------------------------
__global__ void slot_count_kernel(const int32_t* __restrict__ slot_of_row, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[slot_of_row[i]], 1);
}

__global__ void slot_scatter_kernel(const int32_t* __restrict__ slot_of_row, int64_t n,
                                    const int64_t* __restrict__ start, int32_t* __restrict__ cursor,
                                    int32_t* __restrict__ rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = slot_of_row[i];
    const int32_t k = atomicAdd(&cursor[s], 1);
    rows[start[s] + k] = (int32_t)i;
  }
}

__device__ __forceinline__ int64_t find_slot(const uint64_t* __restrict__ keys, int64_t cap_mask, uint64_t k) {
  int64_t s = (int64_t)(fmix64(k) & (uint64_t)cap_mask);
  while (true) {
    const uint64_t cur = keys[s];
    if (cur == k) return s;
    if (cur == dxa::kEmpty) return -1;
    s = (s + 1) & cap_mask;
  }
}

__global__ void probe_count_kernel(const uint64_t* __restrict__ h, const uint8_t* __restrict__ probe_null, int64_t n,
                                   const uint64_t* __restrict__ keys, int64_t cap_mask,
                                   const int32_t* __restrict__ cnt, int32_t* __restrict__ slot_out,
                                   int64_t* __restrict__ out_cnt, int outer) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = -1;
    if (!(probe_null && probe_null[i])) s = find_slot(keys, cap_mask, dxa::fix_key(h[i]));
    slot_out[i] = (int32_t)s;
    int64_t c = s >= 0 ? cnt[s] : 0;
    if (outer && c == 0) c = 1;
    out_cnt[i] = c;
  }
}

__global__ void probe_write_kernel(const int32_t* __restrict__ slot_of_probe, int64_t n,
                                   const int64_t* __restrict__ out_off, const int64_t* __restrict__ start,
                                   const int32_t* __restrict__ cnt, const int32_t* __restrict__ rows,
                                   int64_t* __restrict__ li, int64_t* __restrict__ ri, int outer) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = slot_of_probe[i];
    int64_t o = out_off[i];
    const int32_t c = s >= 0 ? cnt[s] : 0;
    if (c == 0) {
      if (outer) { li[o] = i; ri[o] = -1; }
      continue;
    }
    const int64_t b = start[s];
    for (int32_t k = 0; k < c; ++k) {
      li[o + k] = i;
      ri[o + k] = rows[b + k];
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------------------------
DXA_API int dxa_hash_i64(const int64_t* v, const uint8_t* valid, int64_t n, uint64_t* out, int combine, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hash_i64_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, valid, n, out,
                     combine);
  return (int)hipGetLastError();
}

DXA_API int dxa_hash_f64(const double* v, const uint8_t* valid, int64_t n, uint64_t* out, int combine, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hash_f64_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, valid, n, out,
                     combine);
  return (int)hipGetLastError();
}

DXA_API int dxa_hash_str(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                         int64_t n, uint64_t* out, int combine, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hash_str_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, n, out, combine);
  return (int)hipGetLastError();
}

// keys: [cap] uint64 (filled with 0xFF by the caller), cap power of two.
DXA_API int dxa_table_insert(const uint64_t* h, int64_t n, uint64_t* keys, int64_t cap, int32_t* slot_of_row,
                             void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(table_insert_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, h, n, keys,
                     cap - 1, slot_of_row);
  return (int)hipGetLastError();
}

// counter: [1] int32 zeroed by the caller; rep: [n] int32 filled with INT32_MAX by the caller.
DXA_API int dxa_group_ids(const uint64_t* keys, int64_t cap, const int32_t* slot_of_row, int64_t n,
                          int32_t* gid_of_slot, int32_t* counter, int32_t* gid, int32_t* rep, void* st) {
  hipStream_t s = (hipStream_t)st;
  hipLaunchKernelGGL(table_number_kernel, dim3(dxa_blocks(cap, 256)), dim3(256), 0, s, keys, cap, gid_of_slot,
                     counter);
  if (n > 0)
    hipLaunchKernelGGL(group_gather_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, s, slot_of_row, gid_of_slot, n,
                       gid, rep);
  return (int)hipGetLastError();
}

namespace {
// The group table's initial state, one launch instead of three fills and a memset: keys all-ones (empty), no
// group per slot, counters zero, rep "no row yet".
__global__ __launch_bounds__(256) void group_init_kernel(uint64_t* keys, int64_t cap, int32_t* gid_of_slot,
                                                         int32_t* counter, int32_t* rep, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < cap; i += stride) {
    keys[i] = ~0ull;
    gid_of_slot[i] = -1;
  }
  for (int64_t i = i0; i < n; i += stride) rep[i] = 0x7fffffff;
  if (i0 < 2) counter[i0] = 0;
}
}  // namespace

// dxa_group_build on uninitialised buffers: initialise (one launch), then build.  counter: [2] (ngroups, bad).
DXA_API int dxa_group_build_init(const uint64_t* h, int64_t n, uint64_t* keys, int64_t cap, int32_t* gid_of_slot,
                                 int32_t* counter, int32_t* gid, int32_t* rep, void* st) {
  if (n <= 0) return 0;
  const int64_t work = cap > n ? cap : n;
  const int64_t blocks = (work + 255) / 256;
  hipLaunchKernelGGL(group_init_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                     (hipStream_t)st, keys, cap, gid_of_slot, counter, rep, n);
  hipLaunchKernelGGL(group_build_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, h, n, keys, cap - 1,
                     gid_of_slot, counter, gid, rep);
  return (int)hipGetLastError();
}

// keys: [cap] filled with 0xFF; gid_of_slot: [cap] filled with -1; counter: [1] zeroed; rep: [n] INT32_MAX
DXA_API int dxa_group_build(const uint64_t* h, int64_t n, uint64_t* keys, int64_t cap, int32_t* gid_of_slot,
                            int32_t* counter, int32_t* gid, int32_t* rep, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(group_build_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, h, n, keys, cap - 1,
                     gid_of_slot, counter, gid, rep);
  return (int)hipGetLastError();
}

DXA_API int dxa_verify_i64(const int64_t* v, const uint8_t* valid, const int32_t* gid, const int32_t* rep, int64_t n,
                           int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(verify_i64_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, valid, gid, rep,
                     n, bad);
  return (int)hipGetLastError();
}

DXA_API int dxa_verify_str(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                           const int32_t* gid, const int32_t* rep, int64_t n, int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(verify_str_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, gid, rep, n, bad);
  return (int)hipGetLastError();
}

// op: 0 sum, 1 min, 2 max, 3 count;  vt: 0 int64, 1 double.  out: [ngroups] 8-byte accumulators.
DXA_API int dxa_aggregate(const int32_t* gid, const void* vals, const uint8_t* valid, int64_t n, int32_t ngroups,
                          int32_t op, int32_t vt, void* out, void* st) {
  hipStream_t s = (hipStream_t)st;
  if (ngroups <= 0) return 0;
  if (op == AGG_COUNT) return launch_agg<VT_I64, AGG_COUNT>(gid, vals, valid, n, ngroups, out, s);
  if (vt == VT_I64) {
    if (op == AGG_SUM) return launch_agg<VT_I64, AGG_SUM>(gid, vals, valid, n, ngroups, out, s);
    if (op == AGG_MIN) return launch_agg<VT_I64, AGG_MIN>(gid, vals, valid, n, ngroups, out, s);
    return launch_agg<VT_I64, AGG_MAX>(gid, vals, valid, n, ngroups, out, s);
  }
  if (op == AGG_SUM) return launch_agg<VT_F64, AGG_SUM>(gid, vals, valid, n, ngroups, out, s);
  if (op == AGG_MIN) return launch_agg<VT_F64, AGG_MIN>(gid, vals, valid, n, ngroups, out, s);
  return launch_agg<VT_F64, AGG_MAX>(gid, vals, valid, n, ngroups, out, s);
}

// Fused aggregates: `spec` holds nslots records of 3 int64 (data pointer, validity pointer or 0, value kind) and
// `line_ops` one atomic kind per 8-slot line (kind -1 = unused slot); `out` is int64 [ngroups][8 * nlines], initialised here.
DXA_API int dxa_aggregate_multi(const int32_t* gid, int64_t n, int32_t ngroups, int32_t nslots, const int64_t* spec,
                                int32_t nlines, const int32_t* line_ops, void* out, void* st) {
  if (ngroups <= 0) return 0;
  if (nslots <= 0 || nslots > kMaxAggSlots || nlines * 8 < nslots || nlines > kMaxAggSlots / 8) return 1;
  MultiAggArgs a{};
  a.gid = gid;
  a.n = n;
  a.nslots = nslots;
  a.nlines = nlines;
  a.out = (unsigned long long*)out;
  for (int L = 0; L < nlines; ++L) a.line_op[L] = line_ops[L];
  for (int i = 0; i < nslots; ++i) {
    a.slot[i].data = (const void*)spec[3 * i];
    a.slot[i].valid = (const uint8_t*)spec[3 * i + 1];
    a.slot[i].kind = spec[3 * i + 2];
  }
  hipStream_t s = (hipStream_t)st;
  const int64_t cells = (int64_t)ngroups * nlines * 8;
  hipLaunchKernelGGL(agg_multi_init_kernel, dim3(dxa_blocks(cells, 256)), dim3(256), 0, s, a, ngroups);
  if (n > 0) hipLaunchKernelGGL(agg_multi_kernel, dim3(dxa_blocks(n * 8, 256, 8192)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// Finishing pass of the fused aggregates: every requested aggregate's output column from the [group][slot]
// accumulator rows in ONE launch — counts (held as doubles) to int64, NOT-ed minima back, ordered doubles back to
// doubles, AVG = sum / count, and the "group saw a non-null input" validity — instead of a slice/convert/compare
// chain per aggregate.  dst_data [nreq][ngroups] (int64 or double bits), dst_valid [nreq][ngroups].
constexpr int kMaxFinish = 64;
enum : int { F_COUNT = 0, F_I64 = 1, F_F64 = 2, F_AVG = 3, F_F64_ORD = 4, F_NOT = 8 };

struct FinishArgs {
  const long long* acc;
  int32_t ngroups;
  int32_t stride;
  int32_t nreq;
  int32_t kind[kMaxFinish];
  int32_t pos[kMaxFinish];
  int32_t cnt[kMaxFinish];     // slot of the request's count (-1: none)
  long long* dst;
  uint8_t* valid;
};

__global__ __launch_bounds__(256) void agg_finish_kernel(FinishArgs a) {
  const int64_t total = (int64_t)a.ngroups * a.nreq;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(t / a.ngroups);
    const int64_t g = t - (int64_t)r * a.ngroups;
    const long long* row = a.acc + g * a.stride;
    const int k = a.kind[r];
    long long v = row[a.pos[r]];
    if (k & F_NOT) v = ~v;
    const double c = a.cnt[r] >= 0 ? __longlong_as_double(row[a.cnt[r]]) : 1.0;
    long long o;
    switch (k & 7) {
      case F_COUNT: o = (long long)__longlong_as_double(v); break;
      case F_AVG: o = __double_as_longlong(__longlong_as_double(v) / (c > 1.0 ? c : 1.0)); break;
      case F_F64_ORD: o = v < 0 ? (v ^ 0x7fffffffffffffffll) : v; break;
      default: o = v; break;
    }
    a.dst[t] = o;
    a.valid[t] = c > 0.0 ? 1 : 0;
  }
}

DXA_API int dxa_aggregate_finish(const void* acc, int32_t ngroups, int32_t stride, int32_t nreq, const int32_t* spec,
                                 void* dst, uint8_t* valid, void* st) {
  if (ngroups <= 0 || nreq <= 0) return 0;
  if (nreq > kMaxFinish) return 1;
  FinishArgs a{};
  a.acc = (const long long*)acc;
  a.ngroups = ngroups;
  a.stride = stride;
  a.nreq = nreq;
  for (int r = 0; r < nreq; ++r) {
    a.kind[r] = spec[3 * r];
    a.pos[r] = spec[3 * r + 1];
    a.cnt[r] = spec[3 * r + 2];
  }
  a.dst = (long long*)dst;
  a.valid = valid;
  const int64_t total = (int64_t)ngroups * nreq;
  hipLaunchKernelGGL(agg_finish_kernel, dim3(dxa_blocks(total, 256)), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

DXA_API int dxa_key_cols_size() { return (int)sizeof(KeyCols); }

DXA_API int dxa_hash_multi(const void* args, uint64_t* out, void* st) {
  const KeyCols& a = *(const KeyCols*)args;
  if (a.n <= 0) return 0;
  if (a.ncols <= 0 || a.ncols > kMaxKeyCols) return 1;
  hipLaunchKernelGGL(hash_multi_kernel, dim3(dxa_blocks(a.n, 256)), dim3(256), 0, (hipStream_t)st, a, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_pairs_equal(const void* left, const void* right, const int64_t* li, const int64_t* ri, int64_t m,
                            uint8_t* out, void* st) {
  const KeyCols& L = *(const KeyCols*)left;
  const KeyCols& R = *(const KeyCols*)right;
  if (m <= 0) return 0;
  if (L.ncols <= 0 || L.ncols > kMaxKeyCols || L.ncols != R.ncols) return 1;
  for (int c = 0; c < L.ncols; ++c)
    if (L.c[c].kind != R.c[c].kind) return 1;
  hipLaunchKernelGGL(pairs_equal_kernel, dim3(dxa_blocks(m, 256)), dim3(256), 0, (hipStream_t)st, L, R, li, ri, m,
                     out);
  return (int)hipGetLastError();
}

DXA_API int dxa_verify_multi(const void* args, const int32_t* gid, const int32_t* rep, int32_t* bad, void* st) {
  const KeyCols& a = *(const KeyCols*)args;
  if (a.n <= 0) return 0;
  if (a.ncols <= 0 || a.ncols > kMaxKeyCols) return 1;
  hipLaunchKernelGGL(verify_multi_kernel, dim3(dxa_blocks(a.n, 256)), dim3(256), 0, (hipStream_t)st, a, gid, rep,
                     bad);
  return (int)hipGetLastError();
}

// Final step of merged partial aggregates (distributed / windowed GROUP BY, engine/distagg.py) for many aggregates
// in ONE launch: SUM / MIN / MAX keep their merged data and become NULL where no input row was non-null
// (valid = own validity & count > 0); AVG = sum / max(count, 1) with the same validity.
constexpr int kMaxPartialFinish = 32;
struct PartialFinishReq {
  const long long* data;     // merged value (int64 or double bits)
  const uint8_t* valid;      // its validity (null: all valid)
  const long long* cnt;      // merged count
  long long* out;            // AVG result (double bits); unused for kind 0
  uint8_t* out_valid;
  int32_t kind;              // 0 value-by-count, 1 average
  int32_t pad;
};
struct PartialFinishArgs {
  PartialFinishReq r[kMaxPartialFinish];
  int32_t nreq;
  int64_t n;
};

__global__ __launch_bounds__(256) void partial_finish_kernel(PartialFinishArgs a) {
  const int64_t total = a.n * a.nreq;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(t / a.n);
    const int64_t i = t - (int64_t)q * a.n;
    const PartialFinishReq& r = a.r[q];
    const long long c = r.cnt[i];
    const bool ok = c > 0 && (r.valid == nullptr || r.valid[i] != 0);
    if (r.kind == 1)
      r.out[i] = __double_as_longlong(__longlong_as_double(r.data[i]) / (double)(c > 1 ? c : 1));
    r.out_valid[i] = ok ? 1 : 0;
  }
}

DXA_API int dxa_partial_finish_size() { return (int)sizeof(PartialFinishArgs); }

DXA_API int dxa_partial_finish(const void* args, void* st) {
  const PartialFinishArgs& a = *(const PartialFinishArgs*)args;
  if (a.n <= 0 || a.nreq <= 0) return 0;
  if (a.nreq > kMaxPartialFinish) return 1;
  hipLaunchKernelGGL(partial_finish_kernel, dim3(dxa_blocks(a.n * a.nreq, 256)), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

// Group ids in first-occurrence order (the CPU reference's numbering): the groups' representative rows (their
// first row) are sorted in one workgroup — a bitonic sort of (row << 32 | group) keys in LDS, up to kRenumberMax
// groups — giving each group its rank, then one pass rewrites the row → group map.  Replaces an argsort and four
// indexing launches.
constexpr int kRenumberMax = 4096;

__global__ __launch_bounds__(1024) void renumber_sort_kernel(const int32_t* __restrict__ rep, int32_t ng,
                                                             int32_t* __restrict__ inv, int64_t* __restrict__ rep_out) {
  __shared__ unsigned long long k[kRenumberMax];
  int m = 1;
  while (m < ng) m <<= 1;
  for (int i = threadIdx.x; i < m; i += blockDim.x)
    k[i] = i < ng ? (((unsigned long long)(uint32_t)rep[i]) << 32) | (uint32_t)i : ~0ull;
  __syncthreads();
  for (int size = 2; size <= m; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const unsigned long long a = k[i], b = k[j];
          if ((a > b) == up) { k[i] = b; k[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (int p = threadIdx.x; p < ng; p += blockDim.x) {
    const unsigned long long v = k[p];
    inv[(int32_t)(v & 0xffffffffu)] = p;
    rep_out[p] = (int64_t)(v >> 32);
  }
}

__global__ void renumber_rows_kernel(int32_t* __restrict__ gid, int64_t n, const int32_t* __restrict__ inv) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gid[i] = inv[gid[i]];
}

// Any number of groups over at most kBitmapRows rows: a group's rank is the number of first rows before its own,
// read off a bitmap of first rows held in LDS (64 KiB) and the word-wise exclusive popcount sums (32 KiB).
constexpr int kBitmapWords = 8192;
constexpr int64_t kBitmapRows = (int64_t)kBitmapWords * 64;

__global__ __launch_bounds__(1024) void renumber_bitmap_kernel(const int32_t* __restrict__ rep, int32_t ng,
                                                               int32_t* __restrict__ inv,
                                                               int64_t* __restrict__ rep_out) {
  __shared__ unsigned long long bits[kBitmapWords];
  __shared__ uint32_t pre[kBitmapWords];
  __shared__ uint32_t wsum[16];
  const int t = threadIdx.x;
  for (int w = t; w < kBitmapWords; w += blockDim.x) bits[w] = 0ull;
  __syncthreads();
  for (int g = t; g < ng; g += blockDim.x) {
    const uint32_t r = (uint32_t)rep[g];
    atomicOr(&bits[r >> 6], 1ull << (r & 63));
  }
  __syncthreads();
  // exclusive scan of the words' popcounts: 8 consecutive words per thread, then a block scan of the thread sums
  constexpr int kPer = kBitmapWords / 1024;
  uint32_t local = 0;
  for (int k = 0; k < kPer; ++k) local += (uint32_t)__popcll(bits[t * kPer + k]);
  const int lane = t & 63, wid = t >> 6;
  uint32_t incl = local;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int k = 0; k < (int)(blockDim.x / 64); ++k) {
      const uint32_t v = wsum[k];
      wsum[k] = acc;
      acc += v;
    }
  }
  __syncthreads();
  uint32_t run = wsum[wid] + incl - local;
  for (int k = 0; k < kPer; ++k) {
    pre[t * kPer + k] = run;
    run += (uint32_t)__popcll(bits[t * kPer + k]);
  }
  __syncthreads();
  for (int g = t; g < ng; g += blockDim.x) {
    const uint32_t r = (uint32_t)rep[g];
    const uint32_t w = r >> 6;
    const unsigned long long below = (r & 63) ? (bits[w] & ((1ull << (r & 63)) - 1ull)) : 0ull;
    const int32_t rank = (int32_t)(pre[w] + (uint32_t)__popcll(below));
    inv[g] = rank;
    rep_out[rank] = (int64_t)r;
  }
}

DXA_API int dxa_group_renumber_max() { return kRenumberMax; }
DXA_API int64_t dxa_group_renumber_bitmap_rows() { return kBitmapRows; }

// gid: [n] int32 rewritten in place; rep: [ng] int32 first rows; inv: [ng] int32 scratch; rep_out: [ng] int64
DXA_API int dxa_group_renumber(int32_t* gid, int64_t n, const int32_t* rep, int32_t ng, int32_t* inv,
                               int64_t* rep_out, void* st) {
  if (ng <= 0) return 0;
  hipStream_t s = (hipStream_t)st;
  if (n <= kBitmapRows)
    hipLaunchKernelGGL(renumber_bitmap_kernel, dim3(1), dim3(1024), 0, s, rep, ng, inv, rep_out);
  else if (ng <= kRenumberMax)
    hipLaunchKernelGGL(renumber_sort_kernel, dim3(1), dim3(1024), 0, s, rep, ng, inv, rep_out);
  else
    return 1;
  if (n > 0) hipLaunchKernelGGL(renumber_rows_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, s, gid, n, inv);
  return (int)hipGetLastError();
}

DXA_API int dxa_slot_count(const int32_t* slot_of_row, int64_t n, int32_t* cnt, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(slot_count_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, slot_of_row, n, cnt);
  return (int)hipGetLastError();
}

DXA_API int dxa_slot_scatter(const int32_t* slot_of_row, int64_t n, const int64_t* start, int32_t* cursor,
                             int32_t* rows, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(slot_scatter_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, slot_of_row, n,
                     start, cursor, rows);
  return (int)hipGetLastError();
}

DXA_API int dxa_probe_count(const uint64_t* h, const uint8_t* probe_null, int64_t n, const uint64_t* keys, int64_t cap,
                            const int32_t* cnt, int32_t* slot_out, int64_t* out_cnt, int outer, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(probe_count_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, h, probe_null, n,
                     keys, cap - 1, cnt, slot_out, out_cnt, outer);
  return (int)hipGetLastError();
}

DXA_API int dxa_probe_write(const int32_t* slot_of_probe, int64_t n, const int64_t* out_off, const int64_t* start,
                            const int32_t* cnt, const int32_t* rows, int64_t* li, int64_t* ri, int outer, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(probe_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, slot_of_probe, n,
                     out_off, start, cnt, rows, li, ri, outer);
  return (int)hipGetLastError();
}
