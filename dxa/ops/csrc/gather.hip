// Multi-column row gather for gfx950: `dst_k[i] = src_k[idx[i]]` for up to kMaxCols columns in ONE launch.
//
// A table take (filter, join output, group representative rows, ORDER BY) touches every leaf tensor of every
// column — data, validity, string starts and lengths — with the same row index vector.  Gathering them one
// tensor at a time costs a launch and a framework call per leaf (a 30-leaf IoT row is ~30 launches); here the index
// is read once per row and every column of the launch is served from it.  grid.y walks the columns in groups of
// kColsPerBlock so wide tables still fill the machine; descriptors travel in the kernel argument block (no upload).
// Negative indices count from the end (torch semantics); indices outside [-n, n) produce zero bytes.
#include "dxa_common.h"

namespace {

constexpr int kMaxCols = 48;

struct GatherCol {
  const void* src;
  void* dst;
  int32_t elem;          // 1, 2, 4 or 8 bytes
  int32_t pad;
};

struct GatherArgs {
  GatherCol cols[kMaxCols];
  int32_t ncols;
  int64_t n_src;
  int64_t n_idx;
  const int64_t* idx;
};

template <typename T>
__device__ __forceinline__ void move1(const GatherCol& c, int64_t i, int64_t j, bool ok) {
  reinterpret_cast<T*>(c.dst)[i] = ok ? reinterpret_cast<const T*>(c.src)[j] : T(0);
}

constexpr int kColsPerBlock = 8;

__global__ __launch_bounds__(256) void multi_gather_kernel(const GatherArgs a) {
  const int c0 = blockIdx.y * kColsPerBlock;
  const int c1 = c0 + kColsPerBlock < a.ncols ? c0 + kColsPerBlock : a.ncols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n_idx; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t j = a.idx[i];
    if (j < 0) j += a.n_src;
    const bool ok = j >= 0 && j < a.n_src;
    if (!ok) j = 0;
    for (int c = c0; c < c1; ++c) {
      const GatherCol& col = a.cols[c];
      switch (col.elem) {
        case 8: move1<uint64_t>(col, i, j, ok); break;
        case 4: move1<uint32_t>(col, i, j, ok); break;
        case 2: move1<uint16_t>(col, i, j, ok); break;
        default: move1<uint8_t>(col, i, j, ok); break;
      }
    }
  }
}

}  // namespace

DXA_API int dxa_multi_gather_max_cols() { return kMaxCols; }

// srcs/dsts/elems: ncols entries (ncols <= dxa_multi_gather_max_cols()); every src has n_src elements, every dst
// n_idx elements.
DXA_API int dxa_multi_gather(const void* const* srcs, void* const* dsts, const int32_t* elems, int32_t ncols,
                             int64_t n_src, const int64_t* idx, int64_t n_idx, void* st) {
  if (ncols <= 0 || n_idx <= 0) return 0;
  if (ncols > kMaxCols) return (int)hipErrorInvalidValue;
  GatherArgs a{};
  for (int c = 0; c < ncols; ++c) {
    if (elems[c] != 1 && elems[c] != 2 && elems[c] != 4 && elems[c] != 8) return (int)hipErrorInvalidValue;
    a.cols[c] = GatherCol{srcs[c], dsts[c], elems[c], 0};
  }
  a.ncols = ncols;
  a.n_src = n_src;
  a.n_idx = n_idx;
  a.idx = idx;
  const unsigned gy = (unsigned)((ncols + kColsPerBlock - 1) / kColsPerBlock);
  const int gx = dxa::grid_stride_blocks(n_idx, 256, 2048);
  hipLaunchKernelGGL(multi_gather_kernel, dim3(gx, gy), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}
