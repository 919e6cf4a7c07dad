// Device -> pinned-host copies on the GPU's SDMA engines.
//
// hipMemcpyAsync(DeviceToHost) into pinned memory runs as a shader blit kernel on gfx950 (__amd_rocclr_copyBuffer
// in the kernel trace): the kernel writes host memory over PCIe and holds its CUs for the whole transfer.  The
// passthrough flow moves ~0.7 GB of rendered JSON per batch that way, ~14 ms of blit-kernel time per step competing
// with the LZ4 decode and the parser on the same CUs.  The ROCr async copy API puts the transfer on a DMA engine
// instead; the caller (a host output thread) blocks on its completion signal, after the producing kernels are done.
#include "dxa_common.h"
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

DXA_API int dxa_copy_sdma(void* dst, const void* src, int64_t n) {
  if (n <= 0) return 0;
  hsa_amd_pointer_info_t di{}, si{};
  di.size = sizeof(di);
  si.size = sizeof(si);
  if (hsa_amd_pointer_info(dst, &di, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return -1;
  if (hsa_amd_pointer_info(const_cast<void*>(src), &si, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return -2;
  if (di.type == HSA_EXT_POINTER_TYPE_UNKNOWN || si.type == HSA_EXT_POINTER_TYPE_UNKNOWN) return -3;
  hsa_signal_t sig;
  if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return -4;
  const hsa_status_t st = hsa_amd_memory_async_copy(dst, di.agentOwner, src, si.agentOwner, (size_t)n, 0, nullptr,
                                                    sig);
  if (st != HSA_STATUS_SUCCESS) {
    hsa_signal_destroy(sig);
    return -5;
  }
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) != 0) {
  }
  hsa_signal_destroy(sig);
  return 0;
}
