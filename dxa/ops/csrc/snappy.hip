// Snappy raw-block decoder for gfx950: snappy-compressed Kafka record batches (codec 2 — the planner splits
// snappy-java's xerial stream into its independent raw blocks, each with its exact size in the varint preamble)
// are decompressed in HBM after a compressed H2D copy, like the LZ4 / gzip / zstd batches.
//
// Layout: 16 lanes own one block (4 blocks per wave) and parse the tag chain redundantly on group-uniform state
// (the chain is serial: every tag's position depends on the previous element's length); the lanes split the byte
// work 16 per step — literal runs straight from the compressed input, copies as dst[s + (i mod off)], whose sources
// always precede the copy's own start (an overlapping copy replicates its period without a dependency inside the
// step).  A `s_waitcnt vmcnt(0)` before a copy whose source reaches past the output known complete at the last
// wait makes the group's earlier stores visible (as lz4.hip).  Every length, offset and input position is checked;
// a malformed block stops with a nonzero status, never an out-of-range access.
#include "dxa_common.h"

namespace {

constexpr int SG = 16;                  // lanes per block
constexpr int SWG = 256;                // threads per workgroup: 16 blocks
constexpr int kWaitVm0 = 0xF70;         // s_waitcnt vmcnt(0) (gfx9 encoding)

enum : int32_t { S_OK = 0, S_TRUNC = 1, S_OFFSET = 2, S_OVERFLOW = 3, S_SIZE = 4 };

__device__ __forceinline__ void stores_visible() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(SWG) void snappy_block_kernel(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ comp_off,
                                                           const int32_t* __restrict__ comp_len,
                                                           const uint8_t* __restrict__ kind,
                                                           const int64_t* __restrict__ out_off,
                                                           const int64_t* __restrict__ cap_arr, int64_t nb,
                                                           uint8_t* __restrict__ dst, int64_t* __restrict__ produced,
                                                           int32_t* __restrict__ status) {
  const int64_t b = ((int64_t)blockIdx.x * SWG + threadIdx.x) / SG;
  const int gl = (int)(threadIdx.x & (SG - 1));
  if (b >= nb || kind[b] != 3) return;
  const uint8_t* in = src + comp_off[b];
  const int32_t n = comp_len[b];
  const int64_t cap64 = cap_arr[b];
  uint8_t* out = dst + out_off[b];
  int32_t rc = S_OK;
  if (n < 1 || cap64 < 0 || cap64 > INT32_MAX) rc = S_SIZE;
  // varint preamble: the block's uncompressed length
  int64_t total = 0;
  int32_t ip = 0;
  if (rc == S_OK) {
    int shift = 0;
    bool end = false;
    while (ip < n && ip < 5) {
      const uint32_t x = in[ip++];
      total |= (int64_t)(x & 127) << shift;
      shift += 7;
      if (!(x & 128)) { end = true; break; }
    }
    if (!end || total != cap64) rc = S_SIZE;
  }
  const int32_t cap = (int32_t)cap64;
  int32_t op = 0, done = 0;
  while (rc == S_OK && ip < n) {
    const uint32_t tag = in[ip++];
    const uint32_t k = tag & 3;
    if (k == 0) {
      int32_t len = (int32_t)(tag >> 2) + 1;
      if ((tag >> 2) >= 60) {
        const int nbt = (int)(tag >> 2) - 59;
        if (ip + nbt > n) { rc = S_TRUNC; break; }
        uint32_t v = 0;
        for (int j = 0; j < nbt; ++j) v |= (uint32_t)in[ip + j] << (8 * j);
        ip += nbt;
        if (v >= 0x7fffffffu) { rc = S_OVERFLOW; break; }
        len = (int32_t)v + 1;
      }
      if (len > n - ip) { rc = S_TRUNC; break; }
      if (len > cap - op) { rc = S_OVERFLOW; break; }
      for (int32_t c = gl; c < len; c += SG) out[op + c] = in[ip + c];
      ip += len;
      op += len;
      continue;
    }
    int32_t len, off;
    if (k == 1) {
      if (ip >= n) { rc = S_TRUNC; break; }
      len = (int32_t)((tag >> 2) & 7) + 4;
      off = (int32_t)(((tag >> 5) << 8) | in[ip]);
      ip += 1;
    } else if (k == 2) {
      if (ip + 2 > n) { rc = S_TRUNC; break; }
      len = (int32_t)(tag >> 2) + 1;
      off = (int32_t)((uint32_t)in[ip] | ((uint32_t)in[ip + 1] << 8));
      ip += 2;
    } else {
      if (ip + 4 > n) { rc = S_TRUNC; break; }
      len = (int32_t)(tag >> 2) + 1;
      const uint32_t o = (uint32_t)in[ip] | ((uint32_t)in[ip + 1] << 8) | ((uint32_t)in[ip + 2] << 16) |
                         ((uint32_t)in[ip + 3] << 24);
      if (o > 0x7fffffffu) { rc = S_OFFSET; break; }
      off = (int32_t)o;
      ip += 4;
    }
    if (off == 0 || off > op) { rc = S_OFFSET; break; }
    if (len > cap - op) { rc = S_OVERFLOW; break; }
    const int32_t s = op - off;
    if (s + (len < off ? len : off) > done) {            // source reaches past the visible output
      stores_visible();
      done = op;
    }
    for (int32_t c = gl; c < len; c += SG) out[op + c] = out[s + (c % off)];
    op += len;
  }
  if (rc == S_OK && op != cap) rc = S_SIZE;
  if (gl == 0) {
    status[b] = rc;
    produced[b] = rc == S_OK ? op : 0;
  }
}

}  // namespace

// Decode every kind-3 (snappy raw block) entry of a block table; other kinds are left alone.
DXA_API int dxa_snappy_decode_into(const void* src, const void* comp_off, const void* comp_len, const void* kind,
                                   const void* out_off, const void* cap, int64_t nb, void* dst, void* produced,
                                   void* status, void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(snappy_block_kernel, dim3((unsigned)((nb * SG + SWG - 1) / SWG)), dim3(SWG), 0,
                     (hipStream_t)st, (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len,
                     (const uint8_t*)kind, (const int64_t*)out_off, (const int64_t*)cap, nb, (uint8_t*)dst,
                     (int64_t*)produced, (int32_t*)status);
  return (int)hipGetLastError();
}
