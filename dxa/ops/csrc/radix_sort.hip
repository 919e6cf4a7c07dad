// LSD radix sort of (uint64 key, int64 value) pairs for gfx950 — kernel K14 (ORDER BY, window
// functions, string ranking), plus the order-key builders the SQL layer sorts with.
//
// One pass sorts by one 8-bit digit, stably, in three launches:
//   rs_hist_kernel     each workgroup counts the digits of its 4096-item tile (per-wave LDS histograms);
//   rs_scan_*          exclusive scan of the digit-major count matrix [256 digits][tiles] → where every
//                      (digit, tile) run starts in the output;
//   rs_scatter_kernel  each workgroup ranks its tile stably (64-lane match of equal digits with 8 ballots, running
//                      per-digit counts in LDS across the tile's wave-iterations), stages the tile in LDS in digit
//                      order and writes every digit run out as consecutive addresses.
// Tiles are 256 lanes x 16 items, striped (item = it * 256 + lane), so loads and stores are coalesced and the
// (iteration, wave, lane) order is the index order — which is what makes the ranking stable.  `rs_byte_hist`
// counts all eight bytes of the keys in one read so the driver (dxa/ops/sort.py) skips bytes that are constant
// over the whole input (most passes for small integers, timestamps within a day, row ranks).
#include "dxa_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;    // 4096
constexpr int kRadix = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint32_t digit_of(uint64_t k, int shift) { return (uint32_t)(k >> shift) & 0xffu; }

// lanes of this wave whose digit equals mine (8 ballots over the digit bits)
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool active) {
  uint64_t peers = __ballot(active);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t ones = __ballot(active && bit);
    peers &= bit ? ones : ~ones;
  }
  return active ? peers : 0ull;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = threadIdx.x & 63u;
  return lane ? ((~0ull) >> (64 - lane)) : 0ull;
}

__global__ __launch_bounds__(kThreads) void rs_hist_kernel(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                           int32_t* __restrict__ counts, int64_t ntiles) {
  __shared__ int32_t h[kWaves][kRadix];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  // equal digits of a wave are combined first (8 ballots), so skewed keys cost one LDS add per distinct digit
  // instead of 64 serialised atomics on one counter
#pragma unroll 4
  for (int it = 0; it < kItems; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    const bool active = i < n;
    const uint32_t d = active ? digit_of(keys[i], shift) : 0u;
    const uint64_t peers = match_digit(d, active);
    if (active && (peers & lanemask_lt()) == 0) h[w][d] += __popcll(peers);   // one leader per digit per wave
  }
  __syncthreads();
  for (int d = threadIdx.x; d < kRadix; d += kThreads) {
    int32_t c = 0;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) c += h[q][d];
    counts[(int64_t)d * ntiles + blockIdx.x] = c;
  }
}

// Exclusive scan of m int32 counts into int64 offsets: per-chunk sums, a single-workgroup scan of the chunk sums,
// then each chunk scans itself from its base.
constexpr int kScanChunk = 4096;

__global__ __launch_bounds__(kThreads) void rs_scan_sums_kernel(const int32_t* __restrict__ c, int64_t m,
                                                                int64_t* __restrict__ sums) {
  __shared__ int64_t part[kThreads];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  int64_t s = 0;
  for (int k = threadIdx.x; k < kScanChunk; k += kThreads) {
    const int64_t i = base + k;
    if (i < m) s += c[i];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = part[0];
}

// block-wide exclusive scan of one value per thread (returns the exclusive prefix; *total gets the sum)
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* sh, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
  for (int q = 0; q < kWaves; ++q) {
    if (q < w) wbase += sh[q];
    tot += sh[q];
  }
  __syncthreads();
  *total = tot;
  return wbase + incl - v;
}

__global__ __launch_bounds__(kThreads) void rs_scan_top_kernel(int64_t* __restrict__ sums, int64_t nchunks) {
  __shared__ int64_t sh[kWaves];
  int64_t carry = 0;
  for (int64_t b = 0; b < nchunks; b += kThreads) {
    const int64_t i = b + threadIdx.x;
    const int64_t v = i < nchunks ? sums[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan(v, sh, &tot);
    if (i < nchunks) sums[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kThreads) void rs_scan_chunk_kernel(const int32_t* __restrict__ c, int64_t m,
                                                                 const int64_t* __restrict__ sums,
                                                                 int64_t* __restrict__ out) {
  __shared__ int64_t sh[kWaves];
  const int64_t base = (int64_t)blockIdx.x * kScanChunk;
  int64_t carry = sums[blockIdx.x];
  for (int k = 0; k < kScanChunk; k += kThreads) {
    const int64_t i = base + k + threadIdx.x;
    const int64_t v = i < m ? c[i] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan(v, sh, &tot);
    if (i < m) out[i] = carry + ex;
    carry += tot;
  }
}

// LDS: running per-digit counts, this iteration's per-wave counts, the tile's digit starts, and the staging area
struct ScatterShared {
  int32_t run[kRadix];
  int32_t wcnt[kWaves][kRadix];
  int32_t start[kRadix];
  uint64_t stage[kTile];
};

__global__ __launch_bounds__(kThreads) void rs_scatter_kernel(const uint64_t* __restrict__ keys_in,
                                                              const int64_t* __restrict__ vals_in, int64_t n,
                                                              int shift, const int64_t* __restrict__ offsets,
                                                              int64_t ntiles, uint64_t* __restrict__ keys_out,
                                                              int64_t* __restrict__ vals_out) {
  extern __shared__ uint64_t smem_raw[];
  ScatterShared& S = *reinterpret_cast<ScatterShared*>(smem_raw);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  for (int i = threadIdx.x; i < kRadix; i += kThreads) S.run[i] = 0;
  for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&S.wcnt[0][0])[i] = 0;
  uint64_t k[kItems];
  int32_t pos[kItems];
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    k[it] = i < n ? keys_in[i] : ~0ull;
  }
  __syncthreads();
  // stable local ranks: items are ordered by (iteration, wave, lane)
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    const bool active = i < n;
    const uint32_t d = digit_of(k[it], shift);
    const uint64_t peers = match_digit(d, active);
    const int rank = __popcll(peers & lanemask_lt());
    const bool leader = active && (peers & lanemask_lt()) == 0;
    if (leader) S.wcnt[w][d] = __popcll(peers);
    __syncthreads();
    if (active) {
      int32_t before = S.run[d];
      for (int q = 0; q < w; ++q) before += S.wcnt[q][d];
      pos[it] = before + rank;                     // position among this tile's items with digit d
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < kRadix; dd += kThreads) {
      int32_t add = 0;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) { add += S.wcnt[q][dd]; S.wcnt[q][dd] = 0; }
      S.run[dd] += add;
    }
    __syncthreads();
  }
  // the tile's digit runs start at the exclusive prefix of its per-digit totals
  if (threadIdx.x < 64) {
    // 256 digits by one wave: 4 per lane, then a wave scan
    const int d0 = lane * 4;
    const int32_t c0 = S.run[d0], c1 = S.run[d0 + 1], c2 = S.run[d0 + 2], c3 = S.run[d0 + 3];
    int32_t incl = c0 + c1 + c2 + c3;
    const int32_t own = incl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const int32_t ex = incl - own;
    S.start[d0] = ex;
    S.start[d0 + 1] = ex + c0;
    S.start[d0 + 2] = ex + c0 + c1;
    S.start[d0 + 3] = ex + c0 + c1 + c2;
  }
  __syncthreads();
  // keys: stage in digit order, then write each digit run to consecutive global addresses
  const int64_t valid_items = n - base < kTile ? n - base : kTile;
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    if (i < n) {
      pos[it] += S.start[digit_of(k[it], shift)];
      S.stage[pos[it]] = k[it];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < valid_items; j += kThreads) {
    const uint64_t key = S.stage[j];
    const uint32_t d = digit_of(key, shift);
    keys_out[offsets[(int64_t)d * ntiles + blockIdx.x] + (j - S.start[d])] = key;
  }
  __syncthreads();
  // values: same positions
#pragma unroll
  for (int it = 0; it < kItems; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    if (i < n) S.stage[pos[it]] = (uint64_t)(vals_in ? vals_in[i] : i);
  }
  __syncthreads();
  // the staged keys were overwritten: a digit run's owner is found from the start table (binary search)
  for (int j = threadIdx.x; j < valid_items; j += kThreads) {
    int lo = 0, hi = kRadix - 1;
    while (lo < hi) {                              // last digit whose run starts at or before j
      const int mid = (lo + hi + 1) >> 1;
      if (S.start[mid] <= j) lo = mid; else hi = mid - 1;
    }
    // skip empty runs that share the same start (they are before the owner in digit order)
    vals_out[offsets[(int64_t)lo * ntiles + blockIdx.x] + (j - S.start[lo])] = (int64_t)S.stage[j];
  }
}

// counts of all 8 bytes of every key in one read: hist[byte][256]
__global__ __launch_bounds__(kThreads) void rs_byte_hist_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                                unsigned long long* __restrict__ hist) {
  __shared__ uint32_t h[8][kRadix];
  for (int i = threadIdx.x; i < 8 * kRadix; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const uint64_t k = keys[i];
#pragma unroll
    for (int b = 0; b < 8; ++b) atomicAdd(&h[b][digit_of(k, 8 * b)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8 * kRadix; i += kThreads) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], (unsigned long long)c);
  }
}

// ---- order keys -------------------------------------------------------------------------------------------------

// kind: 0 int64 (two's complement), 1 float64 (IEEE, NaN largest as in Spark), 2 uint64 already ordered.
// Nulls are the caller's (a separate stable pass on the validity byte).  desc flips every bit.
__global__ void order_key_kernel(const uint64_t* __restrict__ in, int64_t n, int kind, int desc,
                                 uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t v = in[i];
    if (kind == 0) {
      v ^= 1ull << 63;
    } else if (kind == 1) {
      if ((v & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) v = 0x7ff8000000000000ull;   // canonical NaN
      if (v == 0x8000000000000000ull) v = 0;                                                 // -0.0 == 0.0
      v = (v >> 63) ? ~v : (v | (1ull << 63));
    }
    out[i] = desc ? ~v : v;
  }
}

// Big-endian 8-byte chunk `chunk` of each string (zero-padded past its end): unsigned comparison of the chunks,
// most significant first, then of the lengths, is the byte-wise (UTF-8 code point) order of the strings.
__global__ void str_chunk_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                 const int32_t* __restrict__ lens, const int64_t* __restrict__ rows, int64_t n,
                                 int chunk, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = rows ? rows[i] : i;
    const int32_t l = lens[r];
    const int32_t off = chunk * 8;
    uint64_t v = 0;
    if (off < l) {
      const uint8_t* s = arena + starts[r] + off;
      const int m = l - off < 8 ? l - off : 8;
      for (int b = 0; b < m; ++b) v |= (uint64_t)s[b] << (56 - 8 * b);
    }
    out[i] = v;
  }
}

}  // namespace

DXA_API int dxa_rs_tile() { return kTile; }

DXA_API int dxa_rs_byte_hist(const uint64_t* keys, int64_t n, unsigned long long* hist, void* st) {
  hipStream_t s = (hipStream_t)st;
  hipError_t e = hipMemsetAsync(hist, 0, sizeof(unsigned long long) * 8 * kRadix, s);
  if (e != hipSuccess) return (int)e;
  if (n <= 0) return 0;
  const int grid = dxa::grid_stride_blocks(n, kThreads, 1024);
  hipLaunchKernelGGL(rs_byte_hist_kernel, dim3(grid), dim3(kThreads), 0, s, keys, n, hist);
  return (int)hipGetLastError();
}

// One stable pass on the byte at `shift`.  `vals_in` may be null (values = input positions).  Scratch: `counts`
// int32[256 * ntiles], `offsets` int64[256 * ntiles], `sums` int64[ceil(256 * ntiles / 4096)].
DXA_API int dxa_rs_pass(const uint64_t* keys_in, const int64_t* vals_in, int64_t n, int shift, int32_t* counts,
                        int64_t* offsets, int64_t* sums, uint64_t* keys_out, int64_t* vals_out, void* st) {
  if (n <= 0) return 0;
  if (shift < 0 || shift > 56 || (shift & 7)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)st;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  const int64_t m = ntiles * kRadix;
  const int64_t nchunks = (m + kScanChunk - 1) / kScanChunk;
  hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)ntiles), dim3(kThreads), 0, s, keys_in, n, shift, counts, ntiles);
  hipLaunchKernelGGL(rs_scan_sums_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, counts, m, sums);
  hipLaunchKernelGGL(rs_scan_top_kernel, dim3(1), dim3(kThreads), 0, s, sums, nchunks);
  hipLaunchKernelGGL(rs_scan_chunk_kernel, dim3((unsigned)nchunks), dim3(kThreads), 0, s, counts, m, sums, offsets);
  hipLaunchKernelGGL(rs_scatter_kernel, dim3((unsigned)ntiles), dim3(kThreads), sizeof(ScatterShared), s, keys_in,
                     vals_in, n, shift, offsets, ntiles, keys_out, vals_out);
  return (int)hipGetLastError();
}

DXA_API int dxa_order_key(const uint64_t* in, int64_t n, int kind, int desc, uint64_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(order_key_kernel, dim3(dxa::grid_stride_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, in, n,
                     kind, desc, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_chunk(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const int64_t* rows,
                          int64_t n, int chunk, uint64_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_chunk_kernel, dim3(dxa::grid_stride_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena,
                     starts, lens, rows, n, chunk, out);
  return (int)hipGetLastError();
}
