// Batched device memcpy / memset: many (src, dst, bytes) segments in ONE launch.
//
// Concatenating tables (window-pane partials, UNION ALL, state snapshots) moves every leaf tensor of every input
// table into an output leaf — with one torch.cat per output tensor (plus a fill per missing validity mask) that is
// two or three launches per column.  Here the host lists the segments in a pinned table (split into chunks of at
// most kChunk bytes so one workgroup owns one chunk), one copy puts the table on the device, and one launch moves
// every byte: 16-byte vector copies when source, destination and length allow it, bytes otherwise.
#include "dxa_common.h"

namespace {

constexpr int64_t kChunk = 64 * 1024;

struct CopyChunk {
  const uint8_t* src;      // null → fill with `fill`
  uint8_t* dst;
  int64_t nbytes;
  int64_t fill;
};

__global__ __launch_bounds__(256) void copy_batch_kernel(const CopyChunk* __restrict__ chunks, int64_t nchunks) {
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const CopyChunk k = chunks[c];
    const int64_t nb = k.nbytes;
    if (k.src == nullptr) {
      const uint8_t f = (uint8_t)k.fill;
      const bool vec = ((reinterpret_cast<uintptr_t>(k.dst) | (uintptr_t)nb) & 15) == 0;
      if (vec) {
        uint32_t w = f | (f << 8) | (f << 16) | ((uint32_t)f << 24);
        const uint4 v = make_uint4(w, w, w, w);
        uint4* d = reinterpret_cast<uint4*>(k.dst);
        for (int64_t i = threadIdx.x; i < nb / 16; i += blockDim.x) d[i] = v;
      } else {
        for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) k.dst[i] = f;
      }
      continue;
    }
    const bool vec = ((reinterpret_cast<uintptr_t>(k.src) | reinterpret_cast<uintptr_t>(k.dst) | (uintptr_t)nb) &
                      15) == 0;
    if (vec) {
      const uint4* s = reinterpret_cast<const uint4*>(k.src);
      uint4* d = reinterpret_cast<uint4*>(k.dst);
      for (int64_t i = threadIdx.x; i < nb / 16; i += blockDim.x) d[i] = s[i];
    } else if (((reinterpret_cast<uintptr_t>(k.src) | reinterpret_cast<uintptr_t>(k.dst) | (uintptr_t)nb) & 7) == 0) {
      const uint64_t* s = reinterpret_cast<const uint64_t*>(k.src);
      uint64_t* d = reinterpret_cast<uint64_t*>(k.dst);
      for (int64_t i = threadIdx.x; i < nb / 8; i += blockDim.x) d[i] = s[i];
    } else {
      for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) k.dst[i] = k.src[i];
    }
  }
}

}  // namespace

DXA_API int dxa_copy_chunk_size() { return (int)sizeof(CopyChunk); }
DXA_API int64_t dxa_copy_chunk_bytes() { return kChunk; }

// chunks: device array of nchunks CopyChunk
DXA_API int dxa_copy_batch(const void* chunks, int64_t nchunks, void* st) {
  if (nchunks <= 0) return 0;
  const unsigned grid = (unsigned)(nchunks < 65535 ? nchunks : 65535);
  hipLaunchKernelGGL(copy_batch_kernel, dim3(grid), dim3(256), 0, (hipStream_t)st, (const CopyChunk*)chunks,
                     nchunks);
  return (int)hipGetLastError();
}
