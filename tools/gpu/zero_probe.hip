// Stand-alone timing of the parser's validity-plane clear (json_parse.hip zero_bytes_kernel, same launch shape)
// against hipMemsetAsync, on an idle GPU: is the kernel slow, or only slow while other streams' kernels run?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void zero_bytes_kernel(uint8_t* __restrict__ p, int64_t nbytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const int64_t head = (int64_t)((16 - (a & 15)) & 15) < nbytes ? (int64_t)((16 - (a & 15)) & 15) : nbytes;
  const int64_t body = (nbytes - head) / 16;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (int64_t i = tid; i < body; i += stride) q[i] = make_uint4(0, 0, 0, 0);
  const int64_t tail0 = head + body * 16;
  if (tid < head) p[tid] = 0;
  if (tid < nbytes - tail0) p[tail0 + tid] = 0;
}

int main() {
  const int64_t sizes[] = {4 << 20, 32 << 20, 33000000};
  uint8_t* p = nullptr;
  if (hipMalloc(&p, 64 << 20) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int64_t nb : sizes) {
    const int64_t body = nb / 16 + 1;
    const int64_t blocks = (body + 255) / 256 < 4096 ? (body + 255) / 256 : 4096;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0, 0);
      for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(zero_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, 0, p, nb);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      hipEventRecord(e0, 0);
      for (int k = 0; k < 20; ++k) hipMemsetAsync(p, 0, nb, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms2 = 0;
      hipEventElapsedTime(&ms2, e0, e1);
      printf("%lld bytes: zero_bytes_kernel %.1f us (%.2f TB/s), hipMemsetAsync %.1f us\n", (long long)nb,
             ms * 1e3 / 20, nb / (ms * 1e-3 / 20) / 1e12, ms2 * 1e3 / 20);
    }
  }
  hipFree(p);
  return 0;
}
