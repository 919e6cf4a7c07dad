// Row-exchange pack / unpack kernels for the RCCL all-to-all (the key shuffle under GROUP BY /
// JOIN / DISTINCT, Spark's Exchange hashpartitioning under CommonProcessorFactory.scala:257-275; X3 all-gathers).
//
// Send side, three launches, one host synchronisation in between (the all-to-all of the send sizes):
//   xchg_hist     per block of kRows rows: row count and string bytes per destination rank (LDS histogram)
//   xchg_scan     one workgroup: exclusive scan of the block histograms (destination-major) → every block's base
//                 row and base byte per destination, plus the [W × (1+S)] send-size matrix the all-to-all needs
//   xchg_scatter  every row straight into the packed [rows × C] int64 send matrix at its destination-ordered,
//                 stable position, its string bytes into the per-leaf send arenas; validity bits folded into
//                 63-bit mask words; each string's offset inside its destination's byte block travels as a column
// Receive side, one launch: xchg_unpack writes every leaf's typed column, validity and string view (start =
// byte base of the row's source rank + the travelled offset), so no scan runs on the receive side.
//
// Layout of a matrix row: [prim data cols | string lens | string offsets | mask words].  Stability matches the
// torch reference path (a stable sort by destination), so both produce identical buffers.
#include "dxa_common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRows = 2048;                // rows per block (8 chunks of 256)
constexpr int kMaxW = 64;                  // ranks
constexpr int kMaxCols = 64;               // prim data columns
constexpr int kMaxValid = 64;              // validity bits
constexpr int kMaxStr = 8;                 // string leaves
constexpr int kMaxExtra = 4;               // extra words per send-size row

// kinds of a prim column (element width)
enum : int32_t { K8 = 0, K4 = 1, K1 = 2, K2 = 3 };

struct XCol {
  const void* data;
  int32_t kind;
  int32_t pad;
};
struct XValid {
  const uint8_t* valid;
  int32_t word;
  int32_t bit;
};
struct XStr {
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
  uint8_t* dst;          // packed send arena of this leaf
};

struct PackArgs {
  const int64_t* dest;   // [n] destination rank (null: every row to rank 0, i.e. a plain pack)
  int64_t n;
  int32_t W;
  int32_t nblocks;
  int32_t ncols;         // prim data columns
  int32_t nvalid;
  int32_t nstr;
  int32_t C;             // matrix width = ncols + 2*nstr + nmask
  int64_t* hist;         // [(1+S)][W][nblocks]: counts (s=0) and bytes; scanned in place to bases
  int64_t* sizes;        // [W][1+S] send sizes
  int64_t* mat;          // [n][C]
  XCol cols[kMaxCols];
  XValid valids[kMaxValid];
  XStr strs[kMaxStr];
  int32_t sizes_stride;  // row stride of `sizes` (>= 1 + nstr)
  int32_t nextra;        // words written after the sizes of every destination row (the layout's validity flags,
  int64_t extra[kMaxExtra];  //   which ride with the send sizes through the size all-to-all)
  int32_t coalesce;      // 1: every leaf's bytes go to ONE arena (strs[*].dst equal), destination-major —
  int32_t pad1;          //   [d0: leaf 0 | leaf 1 | …][d1: …] — so one byte all-to-all moves every string leaf
};

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = threadIdx.x & 63u;
  return lane ? ((~0ull) >> (64 - lane)) : 0ull;
}

__device__ __forceinline__ int32_t str_len(const XStr& s, int64_t i) { return s.lens[i] > 0 ? s.lens[i] : 0; }

typedef uint64_t u64u __attribute__((aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint16_t u16u __attribute__((aligned(1)));

// unaligned 8/4/2/1-byte copies that never touch a byte outside [0, l) of either side
__device__ __forceinline__ void copy_bytes(const uint8_t* s, uint8_t* d, int32_t l) {
  int32_t k = 0;
  for (; k + 8 <= l; k += 8) *(u64u*)(d + k) = *(const u64u*)(s + k);
  if (k + 4 <= l) { *(u32u*)(d + k) = *(const u32u*)(s + k); k += 4; }
  if (k + 2 <= l) { *(u16u*)(d + k) = *(const u16u*)(s + k); k += 2; }
  if (k < l) d[k] = s[k];
}

__global__ __launch_bounds__(kThreads) void xchg_hist_kernel(const PackArgs a) {
  __shared__ unsigned long long h[(1 + kMaxStr) * kMaxW];
  const int S1 = 1 + a.nstr;
  for (int t = threadIdx.x; t < S1 * a.W; t += kThreads) h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRows;
  for (int it = 0; it < kRows / kThreads; ++it) {
    const int64_t i = base + it * kThreads + threadIdx.x;
    if (i < a.n) {
      const int d = a.dest ? (int)a.dest[i] : 0;
      atomicAdd(&h[d], 1ull);
      for (int s = 0; s < a.nstr; ++s) {
        const int32_t l = str_len(a.strs[s], i);
        if (l) atomicAdd(&h[(1 + s) * a.W + d], (unsigned long long)l);
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < S1 * a.W; t += kThreads)
    a.hist[(int64_t)t * a.nblocks + blockIdx.x] = (int64_t)h[t];
}

// One workgroup.  For every s: exclusive scan over (d, b) in destination-major order; sizes[d][s] = Σ_b.
__global__ __launch_bounds__(1024) void xchg_scan_kernel(const PackArgs a) {
  __shared__ int64_t part[1024];
  const int S1 = 1 + a.nstr;
  const int64_t m = (int64_t)a.W * a.nblocks;
  for (int s = 0; s < S1; ++s) {
    int64_t* h = a.hist + (int64_t)s * m;
    // per-destination totals first (a thread per destination)
    for (int d = threadIdx.x; d < a.W; d += blockDim.x) {
      int64_t t = 0;
      for (int b = 0; b < a.nblocks; ++b) t += h[(int64_t)d * a.nblocks + b];
      a.sizes[(int64_t)d * a.sizes_stride + s] = t;
      if (s == 0)
        for (int x = 0; x < a.nextra; ++x) a.sizes[(int64_t)d * a.sizes_stride + S1 + x] = a.extra[x];
    }
    // chunked scan: each thread owns a contiguous run of ceil(m / threads) entries
    const int64_t per = (m + blockDim.x - 1) / blockDim.x;
    const int64_t lo = threadIdx.x * per;
    const int64_t hi = lo + per < m ? lo + per : m;
    int64_t sum = 0;
    for (int64_t k = lo; k < hi; ++k) sum += h[k];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t acc = 0;
      for (int t = 0; t < (int)blockDim.x; ++t) {
        const int64_t v = part[t];
        part[t] = acc;
        acc += v;
      }
    }
    __syncthreads();
    int64_t acc = part[threadIdx.x];
    for (int64_t k = lo; k < hi; ++k) {
      const int64_t v = h[k];
      h[k] = acc;
      acc += v;
    }
    __syncthreads();
  }
}

// Bases of a destination's block are relative to the whole send buffer; the receiver needs a string's offset
// relative to the start of ITS destination's bytes, so the destination base (= the first block's base) is
// subtracted when the offset is written.
__global__ __launch_bounds__(kThreads) void xchg_scatter_kernel(const PackArgs a) {
  __shared__ int64_t wave_tot[kWaves][1 + kMaxStr][kMaxW];
  __shared__ int64_t run[1 + kMaxStr][kMaxW];
  __shared__ int64_t blk[1 + kMaxStr][kMaxW];      // this block's base per (s, d)
  __shared__ int64_t dstart[1 + kMaxStr][kMaxW];   // destination block start per (s, d)
  __shared__ int64_t shift[kMaxStr][kMaxW];        // leaf arena position → coalesced arena position per (s, d)
  const int S1 = 1 + a.nstr;
  const int W = a.W;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)W * a.nblocks;
  for (int t = threadIdx.x; t < S1 * W; t += kThreads) {
    const int s = t / W, d = t % W;
    run[s][d] = 0;
    blk[s][d] = a.hist[(int64_t)s * m + (int64_t)d * a.nblocks + blockIdx.x];
    dstart[s][d] = a.hist[(int64_t)s * m + (int64_t)d * a.nblocks];
    if (s > 0) {
      // coalesced: leaf s of destination d starts after every earlier destination's bytes (all leaves) and the
      // earlier leaves' bytes of d; the sizes matrix [W][sizes_stride] holds the per-(d, leaf) byte counts
      int64_t pos = 0;
      if (a.coalesce) {
        for (int e = 0; e < d; ++e)
          for (int q = 0; q < a.nstr; ++q) pos += a.sizes[(int64_t)e * a.sizes_stride + 1 + q];
        for (int q = 0; q < s - 1; ++q) pos += a.sizes[(int64_t)d * a.sizes_stride + 1 + q];
        pos -= dstart[s][d];
      }
      shift[s - 1][d] = pos;
    }
  }
  const int64_t base = (int64_t)blockIdx.x * kRows;
  const int nmask_base = a.ncols + 2 * a.nstr;
  for (int it = 0; it < kRows / kThreads; ++it) {
    for (int t = threadIdx.x; t < kWaves * S1 * W; t += kThreads) {
      const int w = t / (S1 * W), r = t % (S1 * W);
      wave_tot[w][r / W][r % W] = 0;
    }
    __syncthreads();
    const int64_t i = base + it * kThreads + threadIdx.x;
    const bool act = i < a.n;
    const int d = act ? (a.dest ? (int)a.dest[i] : 0) : -1;
    // per-leaf values live in registers: every index below is a compile-time constant (unrolled, guarded)
    int32_t len[kMaxStr];
#pragma unroll
    for (int s = 0; s < kMaxStr; ++s) len[s] = (s < a.nstr && act) ? str_len(a.strs[s], i) : 0;
    int32_t rank = 0;
    int64_t boff[kMaxStr];
#pragma unroll
    for (int s = 0; s < kMaxStr; ++s) boff[s] = 0;
    // wave-level: one pass per distinct destination among the wave's rows
    uint64_t todo = __ballot(act);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int dd = __shfl(d, leader, 64);
      const uint64_t peers = __ballot(d == dd) & todo;
      if (d == dd) rank = __popcll(peers & lanemask_lt());
      if (lane == leader) wave_tot[wave][0][dd] = __popcll(peers);
#pragma unroll
      for (int s = 0; s < kMaxStr; ++s) {
        if (s >= a.nstr) break;
        int64_t v = (d == dd) ? (int64_t)len[s] : 0;
        int64_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
          const int64_t t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        if (d == dd) boff[s] = incl - v;
        const int64_t tot = __shfl(incl, 63, 64);
        if (lane == leader) wave_tot[wave][1 + s][dd] = tot;
      }
      todo &= ~peers;
    }
    __syncthreads();
    // exclusive prefix over waves (row order = wave order within the chunk), added to the running offsets
    int64_t pre_row = 0;
    int64_t pre_b[kMaxStr];
#pragma unroll
    for (int s = 0; s < kMaxStr; ++s) pre_b[s] = 0;
    if (act) {
      pre_row = run[0][d];
      for (int w = 0; w < wave; ++w) pre_row += wave_tot[w][0][d];
#pragma unroll
      for (int s = 0; s < kMaxStr; ++s) {
        if (s >= a.nstr) break;
        int64_t p = run[1 + s][d];
        for (int w = 0; w < wave; ++w) p += wave_tot[w][1 + s][d];
        pre_b[s] = p;
      }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < S1 * W; t += kThreads) {
      const int s = t / W, dd = t % W;
      int64_t add = 0;
      for (int w = 0; w < kWaves; ++w) add += wave_tot[w][s][dd];
      run[s][dd] += add;
    }
    if (act) {
      const int64_t pos = blk[0][d] + pre_row + rank;
      int64_t* row = a.mat + pos * a.C;
      for (int c = 0; c < a.ncols; ++c) {
        const XCol& col = a.cols[c];
        int64_t v;
        switch (col.kind) {
          case K8: v = ((const int64_t*)col.data)[i]; break;
          case K4: v = (int64_t)((const int32_t*)col.data)[i]; break;
          case K2: v = (int64_t)((const int16_t*)col.data)[i]; break;
          default: v = (int64_t)((const uint8_t*)col.data)[i]; break;
        }
        row[c] = v;
      }
#pragma unroll
      for (int s = 0; s < kMaxStr; ++s) {
        if (s >= a.nstr) break;
        const XStr& st = a.strs[s];
        const int64_t off = blk[1 + s][d] + pre_b[s] + boff[s];      // absolute in this leaf's send arena
        row[a.ncols + s] = (int64_t)st.lens[i];
        row[a.ncols + a.nstr + s] = off - dstart[1 + s][d];           // relative to the destination's bytes
        if (len[s] > 0) copy_bytes(st.arena + st.starts[i], st.dst + off + shift[s][d], len[s]);
      }
      const int nmask = a.C - nmask_base;
      for (int w = 0; w < nmask; ++w) {
        int64_t word = 0;
        for (int v = 0; v < a.nvalid; ++v)       // a null validity pointer: the column has no nulls here
          if (a.valids[v].word == w && (!a.valids[v].valid || a.valids[v].valid[i]))
            word |= (int64_t)1 << a.valids[v].bit;
        row[nmask_base + w] = word;
      }
    }
    __syncthreads();
  }
}

// ---- receive side ----------------------------------------------------------------------------------------------

struct UCol {
  void* out;             // typed output (null for a valid-only leaf)
  uint8_t* valid;        // bool output (null: no validity)
  int32_t kind;          // K8 / K4 / K2 / K1, or -1 for a string leaf
  int32_t mcol;          // matrix column (data or lens)
  int32_t sidx;          // string leaf index (strings)
  int32_t vword;         // mask word (-1: none)
  int32_t vbit;
  int32_t pad;
  int64_t* starts;       // string starts output
};

constexpr int kMaxLeaves = 64;          // keeps UnpackArgs (a by-value kernel argument) under 4 KB

struct UnpackArgs {
  const int64_t* mat;    // received matrix (padded layout when src_row_base differs from row_prefix)
  int64_t n;             // output rows
  int32_t W;
  int32_t nleaf;
  int32_t C;
  int32_t off_col0;      // first string-offset column
  int32_t nstr;
  int32_t mask_col0;
  const int64_t* meta;   // [W+1] row prefix | [W] source row base | [S][W] byte base of source rank's bytes
  UCol leaves[kMaxLeaves];
};

__global__ __launch_bounds__(kThreads) void xchg_unpack_kernel(const UnpackArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const int64_t* row_prefix = a.meta;
  const int64_t* src_base = a.meta + a.W + 1;
  const int64_t* byte_base = a.meta + 2 * a.W + 1;
  int k = 0;
  for (int t = 1; t < a.W; ++t) k = r >= row_prefix[t] ? t : k;
  const int64_t src = src_base[k] + (r - row_prefix[k]);
  const int64_t* row = a.mat + src * a.C;
  for (int li = 0; li < a.nleaf; ++li) {
    const UCol& L = a.leaves[li];
    if (L.valid) L.valid[r] = (uint8_t)((row[a.mask_col0 + L.vword] >> L.vbit) & 1);
    if (L.kind == -1) {
      ((int32_t*)L.out)[r] = (int32_t)row[L.mcol];
      L.starts[r] = byte_base[(int64_t)L.sidx * a.W + k] + row[a.off_col0 + L.sidx];
    } else if (L.out) {
      const int64_t v = row[L.mcol];
      switch (L.kind) {
        case K8: ((int64_t*)L.out)[r] = v; break;
        case K4: ((int32_t*)L.out)[r] = (int32_t)v; break;
        case K2: ((int16_t*)L.out)[r] = (int16_t)v; break;
        default: ((uint8_t*)L.out)[r] = (uint8_t)v; break;
      }
    }
  }
}

}  // namespace

DXA_API int dxa_xchg_limits(int32_t* out) {
  out[0] = kMaxW;
  out[1] = kMaxCols;
  out[2] = kMaxValid;
  out[3] = kMaxStr;
  out[4] = kMaxLeaves;
  out[5] = kRows;
  out[6] = (int32_t)sizeof(PackArgs);
  out[7] = (int32_t)sizeof(UnpackArgs);
  out[8] = kMaxExtra;
  return 0;
}

// Phase 1 (before the size exchange): histograms + scan → hist bases, sizes.
DXA_API int dxa_xchg_plan(const void* args, void* stream) {
  const PackArgs& a = *(const PackArgs*)args;
  // also for n == 0: the (single) block writes the zero histogram the scan reads
  hipLaunchKernelGGL(xchg_hist_kernel, dim3(a.nblocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  hipLaunchKernelGGL(xchg_scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// Phase 2 (after the sizes are known on the host and the send buffers allocated): scatter.
DXA_API int dxa_xchg_scatter(const void* args, void* stream) {
  const PackArgs& a = *(const PackArgs*)args;
  if (a.n > 0)
    hipLaunchKernelGGL(xchg_scatter_kernel, dim3(a.nblocks), dim3(kThreads), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

DXA_API int dxa_xchg_unpack(const void* args, void* stream) {
  const UnpackArgs& a = *(const UnpackArgs*)args;
  if (a.n > 0)
    hipLaunchKernelGGL(xchg_unpack_kernel, dim3((unsigned)((a.n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
