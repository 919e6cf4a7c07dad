// Runtime code generation for fused expression kernels (dxa/engine/jit.py): hipRTC compiles generated HIP C++
// for gfx950 and the module API loads and launches it on torch's streams.  Exported through this library (not
// ctypes straight into libamdhip64) so the launch goes through the same HIP runtime instance torch uses.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DXA_API extern "C" __attribute__((visibility("default")))

// Compile `src` (kernel `name`) for `arch`.  On success *code/*size hold a malloc'd code object (free with
// dxa_rtc_free).  The compiler log (errors and warnings) is copied into `log` (NUL-terminated, truncated to cap).
DXA_API int dxa_rtc_compile(const char* src, const char* name, const char* arch, const char* extra_opt,
                            void** code, int64_t* size, char* log, int64_t log_cap) {
  *code = nullptr;
  *size = 0;
  if (log_cap > 0) log[0] = 0;
  hiprtcProgram prog;
  hiprtcResult r = hiprtcCreateProgram(&prog, src, name, 0, nullptr, nullptr);
  if (r != HIPRTC_SUCCESS) return (int)r + 1000;
  char archopt[64];
  snprintf(archopt, sizeof archopt, "--offload-arch=%s", arch);
  const char* opts[4] = {archopt, "-O3", "-std=c++17", extra_opt};
  const int nopt = (extra_opt && extra_opt[0]) ? 4 : 3;
  r = hiprtcCompileProgram(prog, nopt, opts);
  size_t lsz = 0;
  if (hiprtcGetProgramLogSize(prog, &lsz) == HIPRTC_SUCCESS && lsz > 1 && log_cap > 1) {
    char* tmp = (char*)malloc(lsz);
    if (tmp && hiprtcGetProgramLog(prog, tmp) == HIPRTC_SUCCESS) {
      const size_t m = (size_t)log_cap - 1 < lsz ? (size_t)log_cap - 1 : lsz;
      memcpy(log, tmp, m);
      log[m] = 0;
    }
    free(tmp);
  }
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return (int)r + 1000;
  }
  size_t csz = 0;
  r = hiprtcGetCodeSize(prog, &csz);
  if (r == HIPRTC_SUCCESS) {
    void* buf = malloc(csz);
    r = buf ? hiprtcGetCode(prog, (char*)buf) : HIPRTC_ERROR_OUT_OF_MEMORY;
    if (r == HIPRTC_SUCCESS) {
      *code = buf;
      *size = (int64_t)csz;
    } else {
      free(buf);
    }
  }
  hiprtcDestroyProgram(&prog);
  return r == HIPRTC_SUCCESS ? 0 : (int)r + 1000;
}

DXA_API void dxa_rtc_free(void* p) { free(p); }

// hipRTC version (major * 1000 + minor): part of the disk cache key of compiled code objects.
DXA_API int dxa_rtc_version() {
  int major = 0, minor = 0;
  if (hiprtcVersion(&major, &minor) != HIPRTC_SUCCESS) return -1;
  return major * 1000 + minor;
}

// The fixed compile options of dxa_rtc_compile (before `extra_opt`), for the cache key.
DXA_API const char* dxa_rtc_options() { return "-O3 -std=c++17"; }

DXA_API int dxa_module_load(const void* image, void** module) {
  return (int)hipModuleLoadData(reinterpret_cast<hipModule_t*>(module), image);
}

DXA_API int dxa_module_function(void* module, const char* name, void** fn) {
  return (int)hipModuleGetFunction(reinterpret_cast<hipFunction_t*>(fn), (hipModule_t)module, name);
}

// `params`: array of pointers to each kernel argument's value (hipModuleLaunchKernel convention).
DXA_API int dxa_module_launch(void* fn, uint32_t grid, uint32_t block, void* stream, void** params) {
  return (int)hipModuleLaunchKernel((hipFunction_t)fn, grid, 1, 1, block, 1, 1, 0, (hipStream_t)stream, params,
                                    nullptr);
}
