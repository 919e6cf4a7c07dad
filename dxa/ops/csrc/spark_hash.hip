// Spark SQL hash(): Murmur3_x86_32 chained over the arguments with seed 42 (HashExpression / Murmur3Hash,
// org.apache.spark.sql.catalyst.expressions.hash.scala).  One lane per row; each call folds ONE column into the
// running per-row hash, so a multi-argument hash() is one launch per argument over the same int32 state.
//   * int / date / boolean: hashInt;  long / timestamp: hashLong;  float: hashInt(floatToIntBits), -0.0 → 0;
//     double: hashLong(doubleToLongBits), -0.0 → 0 (NaN canonical, as Java's *ToIntBits / *ToLongBits);
//   * string: hashUnsafeBytes — 4-byte little-endian words, then each tail byte as a SIGNED int (Spark's variant,
//     not the reference Murmur3 tail);
//   * a null argument leaves the row's hash unchanged.
#include "dxa_common.h"

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  return k1 * 0x1b873593u;
}
__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t fmix(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  return h1 ^ (h1 >> 16);
}
__device__ __forceinline__ uint32_t hash_int(uint32_t v, uint32_t seed) { return fmix(mix_h1(seed, mix_k1(v)), 4); }
__device__ __forceinline__ uint32_t hash_long(uint64_t v, uint32_t seed) {
  const uint32_t h1 = mix_h1(seed, mix_k1((uint32_t)v));
  return fmix(mix_h1(h1, mix_k1((uint32_t)(v >> 32))), 8);
}

// kind: 0 int32-valued (int64 storage), 1 long, 2 double, 3 float (stored as double), 4 bool (uint8)
__global__ __launch_bounds__(256) void spark_hash_fixed_kernel(const void* __restrict__ data, int kind,
                                                               const uint8_t* __restrict__ valid, int64_t n,
                                                               int32_t* __restrict__ h) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (valid && !valid[i])) return;
  const uint32_t seed = (uint32_t)h[i];
  uint32_t out;
  if (kind == 4) {
    out = hash_int(reinterpret_cast<const uint8_t*>(data)[i] ? 1u : 0u, seed);
  } else if (kind == 0) {
    out = hash_int((uint32_t)reinterpret_cast<const int64_t*>(data)[i], seed);
  } else if (kind == 1) {
    out = hash_long((uint64_t)reinterpret_cast<const int64_t*>(data)[i], seed);
  } else {
    double d = reinterpret_cast<const double*>(data)[i];
    if (kind == 3) {
      float f = (float)d;
      if (f == 0.0f) f = 0.0f;                                   // -0.0f → 0
      uint32_t bits = __float_as_uint(f);
      if (f != f) bits = 0x7fc00000u;                            // floatToIntBits canonical NaN
      out = hash_int(bits, seed);
    } else {
      if (d == 0.0) d = 0.0;
      uint64_t bits = (uint64_t)__double_as_longlong(d);
      if (d != d) bits = 0x7ff8000000000000ull;                  // doubleToLongBits canonical NaN
      out = hash_long(bits, seed);
    }
  }
  h[i] = (int32_t)out;
}

__global__ __launch_bounds__(256) void spark_hash_str_kernel(const uint8_t* __restrict__ arena,
                                                             const int64_t* __restrict__ starts,
                                                             const int32_t* __restrict__ lens,
                                                             const uint8_t* __restrict__ valid, int64_t n,
                                                             int32_t* __restrict__ h) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (valid && !valid[i])) return;
  const uint8_t* s = arena + starts[i];
  const int32_t len = lens[i];
  uint32_t h1 = (uint32_t)h[i];
  const int32_t aligned = len - (len & 3);
  for (int32_t k = 0; k < aligned; k += 4)
    h1 = mix_h1(h1, mix_k1((uint32_t)s[k] | ((uint32_t)s[k + 1] << 8) | ((uint32_t)s[k + 2] << 16) |
                           ((uint32_t)s[k + 3] << 24)));
  for (int32_t k = aligned; k < len; ++k) h1 = mix_h1(h1, mix_k1((uint32_t)(int32_t)(int8_t)s[k]));
  h[i] = (int32_t)fmix(h1, (uint32_t)len);
}

}  // namespace

DXA_API int dxa_spark_hash_fixed(const void* data, int32_t kind, const uint8_t* valid, int64_t n, int32_t* h,
                                 void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(spark_hash_fixed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     data, kind, valid, n, h);
  return (int)hipGetLastError();
}

DXA_API int dxa_spark_hash_str(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                               int64_t n, int32_t* h, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(spark_hash_str_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     arena, starts, lens, valid, n, h);
  return (int)hipGetLastError();
}
