// Shared device helpers for the dxa gfx950 kernels.
//
// Everything here is written for CDNA4 (wave64): launch geometry is in multiples of 64 lanes, wave-level
// reductions use 64-wide shuffles / 64-bit ballots, and inter-workgroup data only crosses kernel boundaries
// (no in-launch hand-offs), so no release/acquire protocol is needed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DXA_API extern "C" __attribute__((visibility("default")))

namespace dxa {

constexpr int kWave = 64;
constexpr uint64_t kSeed = 0x5bd1e9955bd1e995ull;
constexpr uint64_t kGold = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kNullHash = 0x6e756c6c6e756c6cull;   // "nullnull"
constexpr uint64_t kEmpty = 0xFFFFFFFFFFFFFFFFull;      // empty hash-table slot

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__host__ __device__ __forceinline__ uint64_t hash_i64(uint64_t v) { return fmix64(v ^ kSeed); }

__host__ __device__ __forceinline__ uint64_t hash_combine(uint64_t acc, uint64_t h) {
  return fmix64(acc ^ (h + kGold + (acc << 6) + (acc >> 2)));
}

// Never let a real key collide with the empty-slot sentinel.
__host__ __device__ __forceinline__ uint64_t fix_key(uint64_t h) { return h == kEmpty ? (kEmpty - 1) : h; }

// Unaligned little-endian fetch of n bytes (1..8) starting at p: one or two aligned 8-byte loads and a funnel shift
// instead of n byte loads.  Only aligned words that hold at least one of the n bytes are read, so every load stays
// inside the allocation that holds the bytes (allocations are at least 8-byte aligned).
__device__ __forceinline__ uint64_t load_le(const uint8_t* p, int n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t o = (uint32_t)(a & 7u);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(a - o);
  uint64_t v = w[0] >> (8u * o);
  if (o + (uint32_t)n > 8u) v |= w[1] << (64u - 8u * o);
  return n < 8 ? v & ((1ull << (8 * n)) - 1ull) : v;
}

__device__ __forceinline__ uint64_t hash_bytes(const uint8_t* p, int64_t len) {
  uint64_t h = kSeed ^ ((uint64_t)len * kGold);
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) h = fmix64(h ^ load_le(p + i, 8));
  if (i < len) h = fmix64(h ^ load_le(p + i, (int)(len - i)));
  return fmix64(h ^ (uint64_t)len);
}

// Byte i (0..15) of a 16-byte register window.  Written as a select between two 64-bit halves plus a shift: the
// "pick one of four dwords" form is rewritten by the compiler into a dynamically indexed private array, which it
// then places in LDS or scratch (bank-conflicting per-lane traffic on every byte).
__device__ __forceinline__ uint32_t window_byte(const uint4& w, uint32_t i) {
  const uint64_t lo = ((uint64_t)w.y << 32) | w.x;
  const uint64_t hi = ((uint64_t)w.w << 32) | w.z;
  const uint64_t x = (i & 8u) ? hi : lo;
  return (uint32_t)(x >> ((i & 7u) * 8u)) & 0xffu;
}

// FNV-1a 64 — used for JSON key names (matched against host-computed schema hashes).
__host__ __device__ __forceinline__ uint64_t fnv1a_step(uint64_t h, uint32_t c) {
  return (h ^ (uint64_t)c) * 0x100000001b3ull;
}
constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull;

__host__ __device__ __forceinline__ int grid_stride_blocks(int64_t n, int block, int cap = 256 * 16) {
  int64_t b = (n + block - 1) / block;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

// Civil date → days since 1970-01-01 (proleptic Gregorian).
__host__ __device__ __forceinline__ int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

}  // namespace dxa

inline int dxa_blocks(int64_t n, int block, int cap = 256 * 16) {
  int64_t b = (n + block - 1) / block;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}
