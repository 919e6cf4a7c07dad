// Event-time statistics of a batch in ONE launch (engine/windows.py: a window pane's time span and the late-event
// check): min and max of the valid timestamps, the valid count and the count of valid timestamps >= E.  A
// grid-stride pass reduces per workgroup (wave shuffles + LDS), and the last workgroup to finish (a ticket counter
// that it resets to zero for the next launch) folds the per-workgroup partials — no zero-fill launch, no second
// kernel.  The caller reads the 4 results back with one copy.
#include "dxa_common.h"

namespace {

constexpr int kBlocks = 1024;
constexpr int kThreads = 256;
constexpr int kMaxLens = 32;

struct Stat {
  long long mn, mx, cnt, keep, lens;
};

// string-length arrays whose total the pane's compaction needs (summed in the same pass: no concatenation, no
// separate reduction launch)
struct LensArgs {
  const int32_t* p[kMaxLens];
  int64_t n[kMaxLens];
  int32_t count;
};

__device__ __forceinline__ Stat combine(Stat a, Stat b) {
  Stat r;
  r.mn = a.mn < b.mn ? a.mn : b.mn;
  r.mx = a.mx > b.mx ? a.mx : b.mx;
  r.cnt = a.cnt + b.cnt;
  r.keep = a.keep + b.keep;
  r.lens = a.lens + b.lens;
  return r;
}

__device__ __forceinline__ Stat wave_reduce(Stat s) {
  for (int o = 32; o > 0; o >>= 1) {
    Stat t;
    t.mn = __shfl_down(s.mn, o, 64);
    t.mx = __shfl_down(s.mx, o, 64);
    t.cnt = __shfl_down(s.cnt, o, 64);
    t.keep = __shfl_down(s.keep, o, 64);
    t.lens = __shfl_down(s.lens, o, 64);
    s = combine(s, t);
  }
  return s;
}

__global__ __launch_bounds__(kThreads) void ts_stats_kernel(const int64_t* __restrict__ ts,
                                                            const uint8_t* __restrict__ valid, int64_t n,
                                                            int64_t E, const LensArgs la,
                                                            long long* __restrict__ part,
                                                            unsigned int* __restrict__ ticket,
                                                            long long* __restrict__ out) {
  const long long BIG = 0x7fffffffffffffffll;
  Stat s{BIG, -BIG, 0, 0, 0};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (valid && !valid[i]) continue;
    const long long t = ts[i];
    s.mn = t < s.mn ? t : s.mn;
    s.mx = t > s.mx ? t : s.mx;
    s.cnt += 1;
    s.keep += t >= E ? 1 : 0;
  }
  for (int a = 0; a < la.count; ++a)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < la.n[a]; i += stride) s.lens += la.p[a][i];
  s = wave_reduce(s);
  __shared__ Stat w[kThreads / 64];
  __shared__ bool last;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) w[wid] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    Stat b = w[0];
    for (int k = 1; k < (int)(blockDim.x / 64); ++k) b = combine(b, w[k]);
    long long* p = part + 5 * blockIdx.x;
    p[0] = b.mn;
    p[1] = b.mx;
    p[2] = b.cnt;
    p[3] = b.keep;
    p[4] = b.lens;
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the last workgroup folds the partials in parallel: one partial per thread, then the same wave / LDS reduction
  Stat r{BIG, -BIG, 0, 0, 0};
  for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
    const long long* p = part + 5 * b;
    Stat x{__hip_atomic_load(&p[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
           __hip_atomic_load(&p[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
           __hip_atomic_load(&p[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
           __hip_atomic_load(&p[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
           __hip_atomic_load(&p[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
    r = combine(r, x);
  }
  r = wave_reduce(r);
  __syncthreads();                                         // w[] is reused
  if (lane == 0) w[wid] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    Stat b = w[0];
    for (int k = 1; k < (int)(blockDim.x / 64); ++k) b = combine(b, w[k]);
    out[0] = b.mn;
    out[1] = b.mx;
    out[2] = b.cnt;
    out[3] = b.keep;
    if (la.count) out[4] = b.lens;
    atomicExch(ticket, 0u);                                // ready for the next launch (stream-ordered)
  }
}

}  // namespace

DXA_API int dxa_ts_stats_scratch_bytes() { return kBlocks * 5 * 8 + 64; }
DXA_API int dxa_ts_stats_max_lens() { return kMaxLens; }

// scratch: dxa_ts_stats_scratch_bytes() bytes, zero-initialised once by the caller and reused launch after launch
// on one stream.  out: [4] int64 = min, max, valid count, count(valid & ts >= E); with nlens > 0 string-length
// arrays (int32 lens_ptrs[k] of lens_n[k] entries, host arrays of pointers / counts) a fifth word, their total.
DXA_API int dxa_ts_stats(const int64_t* ts, const uint8_t* valid, int64_t n, int64_t E, void* scratch,
                         long long* out, void* st) {
  LensArgs la{};
  long long* part = (long long*)scratch;
  unsigned int* ticket = (unsigned int*)((char*)scratch + kBlocks * 5 * 8);
  int64_t blocks = (n + kThreads * 4 - 1) / (kThreads * 4);
  if (blocks > kBlocks) blocks = kBlocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ts_stats_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)st, ts, valid, n, E,
                     la, part, ticket, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_ts_stats_lens(const int64_t* ts, const uint8_t* valid, int64_t n, int64_t E, const int64_t* lens_ptrs,
                              const int64_t* lens_n, int32_t nlens, void* scratch, long long* out, void* st) {
  if (nlens < 0 || nlens > kMaxLens) return (int)hipErrorInvalidValue;
  LensArgs la{};
  int64_t most = n;
  for (int k = 0; k < nlens; ++k) {
    la.p[k] = (const int32_t*)lens_ptrs[k];
    la.n[k] = lens_n[k];
    most = lens_n[k] > most ? lens_n[k] : most;
  }
  la.count = nlens;
  long long* part = (long long*)scratch;
  unsigned int* ticket = (unsigned int*)((char*)scratch + kBlocks * 5 * 8);
  int64_t blocks = (most + kThreads * 4 - 1) / (kThreads * 4);
  if (blocks > kBlocks) blocks = kBlocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ts_stats_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, (hipStream_t)st, ts, valid, n, E,
                     la, part, ticket, out);
  return (int)hipGetLastError();
}
