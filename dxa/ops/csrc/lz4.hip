// LZ4 block decoder for gfx950: compressed ingest (LZ4-frame event batches, Kafka compression codec 3) is
// decompressed in HBM after a compressed H2D copy, so PCIe carries ~2.5x fewer bytes per event.
//
// One lane owns one independent block (the frame producer uses 16 KiB blocks, so a 1 GB batch is ~70 K lanes =
// ~1.1 K waves, enough to keep every CU latency-hidden).  A lane runs the sequential LZ4 state machine:
//   * input bytes come through a 16-byte register window (one global_load_dwordx4 per 16 compressed bytes);
//   * output bytes are packed into a 16-byte register accumulator and flushed with aligned 16-B nontemporal
//     stores — only the unaligned head and the tail of a block go out as single bytes (blocks are disjoint);
//   * match sources are read back from the accumulator (offset < 16 bytes behind) or through a second 16-byte
//     window over already-flushed output (same-lane program order makes the flushed bytes visible).
// A size pass (no stores) serves frames whose blocks do not carry decompressed sizes.
#include "dxa_common.h"

namespace {

struct InWin {
  const uint8_t* base;
  uintptr_t wb;
  uint4 w;
  __device__ __forceinline__ uint32_t at(int64_t q) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(base + q);
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != wb) {
      wb = b;
      w = *reinterpret_cast<const uint4*>(b);
    }
    return dxa::window_byte(w, (uint32_t)(a - b));
  }
};

struct OutBuf {
  uint8_t* p;
  int64_t len;
  int head;                 // bytes written singly until p + len is 16-B aligned
  int nacc;
  uint64_t a0, a1;
  uintptr_t wb;             // read-back window over flushed output
  uint4 w;

  __device__ __forceinline__ void init(uint8_t* dst) {
    p = dst; len = 0; nacc = 0; a0 = a1 = 0; wb = 0;
    head = (int)((16 - ((uintptr_t)dst & 15)) & 15);
  }
  __device__ __forceinline__ void put(uint32_t c) {
    if (len < head) {
      p[len] = (uint8_t)c;
      wb = 0;                                   // a cached window may cover this byte
    } else {
      if (nacc < 8) a0 |= (uint64_t)c << (8 * nacc);
      else a1 |= (uint64_t)c << (8 * (nacc - 8));
      if (++nacc == 16) {
        uint64_t* q = reinterpret_cast<uint64_t*>(p + len - 15);
        __builtin_nontemporal_store(a0, q);
        __builtin_nontemporal_store(a1, q + 1);
        a0 = a1 = 0;
        nacc = 0;
      }
    }
    ++len;
  }
  // byte at output position q (< len)
  __device__ __forceinline__ uint32_t get(int64_t q) {
    const int64_t acc0 = len - nacc;
    if (q >= acc0 && len >= head) {
      const int k = (int)(q - acc0);
      return (uint32_t)(((k < 8) ? (a0 >> (8 * k)) : (a1 >> (8 * (k - 8)))) & 0xff);
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + q);
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != wb) {
      wb = b;
      asm volatile("" ::: "memory");            // keep the load after this lane's earlier stores (aliasing types)
      w = *reinterpret_cast<const uint4*>(b);
    }
    return dxa::window_byte(w, (uint32_t)(a - b));
  }
  __device__ __forceinline__ void finish() {
    uint8_t* q = p + len - nacc;
    for (int k = 0; k < nacc; ++k) q[k] = (uint8_t)((k < 8 ? a0 >> (8 * k) : a1 >> (8 * (k - 8))) & 0xff);
  }
};

enum : int32_t { LZ_OK = 0, LZ_TRUNC = 1, LZ_OFFSET = 2, LZ_OVERFLOW = 3, LZ_SIZE = 4 };

// Walk one block's sequences.  WRITE=false: count output bytes only.
template <bool WRITE>
__device__ int32_t run_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t& produced) {
  InWin in{src, 0, make_uint4(0, 0, 0, 0)};
  OutBuf out;
  if (WRITE) out.init(dst);
  int64_t ip = 0, op = 0;
  while (ip < n) {
    const uint32_t token = in.at(ip++);
    int64_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do { if (ip >= n) return LZ_TRUNC; b = in.at(ip++); lit += b; } while (b == 255);
    }
    if (lit > n - ip) return LZ_TRUNC;
    if (lit > cap - op) return LZ_OVERFLOW;
    if (WRITE) for (int64_t k = 0; k < lit; ++k) out.put(in.at(ip + k));
    ip += lit;
    op += lit;
    if (ip >= n) break;
    if (n - ip < 2) return LZ_TRUNC;
    const int64_t off = (int64_t)in.at(ip) | ((int64_t)in.at(ip + 1) << 8);
    ip += 2;
    if (off == 0 || off > op) return LZ_OFFSET;
    int64_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do { if (ip >= n) return LZ_TRUNC; b = in.at(ip++); ml += b; } while (b == 255);
    }
    ml += 4;
    if (ml > cap - op) return LZ_OVERFLOW;
    if (WRITE) {
      const int64_t s = op - off;
      if (off == 1) {
        const uint32_t c = out.get(s);
        for (int64_t k = 0; k < ml; ++k) out.put(c);
      } else {
        for (int64_t k = 0; k < ml; ++k) out.put(out.get(s + k));
      }
    }
    op += ml;
  }
  if (WRITE) out.finish();
  produced = op;
  return LZ_OK;
}

__global__ __launch_bounds__(256) void lz4_sizes_kernel(const uint8_t* __restrict__ src,
                                                        const int64_t* __restrict__ comp_off,
                                                        const int32_t* __restrict__ comp_len,
                                                        const uint8_t* __restrict__ stored, int64_t nb,
                                                        int64_t max_block, int64_t* __restrict__ out_len,
                                                        int32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  if (stored[b]) { out_len[b] = comp_len[b]; status[b] = LZ_OK; return; }
  int64_t produced = 0;
  const int32_t rc = run_block<false>(src + comp_off[b], comp_len[b], nullptr, max_block, produced);
  out_len[b] = rc == LZ_OK ? produced : 0;
  status[b] = rc;
}

__global__ __launch_bounds__(256) void lz4_decode_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ comp_off,
                                                         const int32_t* __restrict__ comp_len,
                                                         const uint8_t* __restrict__ stored,
                                                         const int64_t* __restrict__ out_off,
                                                         const int64_t* __restrict__ out_len, int64_t nb,
                                                         uint8_t* dst, int32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint8_t* s = src + comp_off[b];
  const int64_t n = comp_len[b];
  uint8_t* d = dst + out_off[b];
  const int64_t cap = out_len[b];
  if (stored[b]) {
    if (n != cap) { status[b] = LZ_SIZE; return; }
    InWin in{s, 0, make_uint4(0, 0, 0, 0)};
    OutBuf out;
    out.init(d);
    for (int64_t k = 0; k < n; ++k) out.put(in.at(k));
    out.finish();
    status[b] = LZ_OK;
    return;
  }
  int64_t produced = 0;
  int32_t rc = run_block<true>(s, n, d, cap, produced);
  if (rc == LZ_OK && produced != cap) rc = LZ_SIZE;
  status[b] = rc;
}

}  // namespace

DXA_API int dxa_lz4_block_sizes(const void* src, const void* comp_off, const void* comp_len, const void* stored,
                                int64_t nb, int64_t max_block, void* out_len, void* status, void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(lz4_sizes_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)stored,
                     nb, max_block, (int64_t*)out_len, (int32_t*)status);
  return (int)hipGetLastError();
}

DXA_API int dxa_lz4_decode(const void* src, const void* comp_off, const void* comp_len, const void* stored,
                           const void* out_off, const void* out_len, int64_t nb, void* dst, void* status, void* st) {
  if (nb <= 0) return 0;
  // 64-lane blocks: lanes are long-running and independent, so small workgroups spread blocks over all CUs
  hipLaunchKernelGGL(lz4_decode_kernel, dim3((unsigned)((nb + 63) / 64)), dim3(64), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)stored,
                     (const int64_t*)out_off, (const int64_t*)out_len, nb, (uint8_t*)dst, (int32_t*)status);
  return (int)hipGetLastError();
}
