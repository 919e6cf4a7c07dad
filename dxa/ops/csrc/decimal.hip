// Exact Spark DecimalType(p, s) text conversions on device (input schemas are Spark DataType JSON,
// SchemaFile.scala:25, and SimulatedData emits decimal fields, DataGen.cs:162,195).
//
// Storage (dxa/engine/decimal.py): the unscaled integer per row — one int64 for p ≤ 18, (lo, hi) int64 pairs for
// p ≤ 38.  Two kernels, one lane per row (decimal texts are at most ~48 bytes):
//   * dec_from_text: JSON number tokens / CAST(string AS DECIMAL) → unscaled at scale s, HALF_UP on the first
//     dropped digit (java.math.BigDecimal.setScale(s, ROUND_HALF_UP)), NULL when |v| ≥ 10^p or the text is not a
//     number ([+-]digits[.digits][e[+-]digits], as BigDecimal(String) accepts);
//   * dec_to_text: Java BigDecimal.toString of the value (plain digits with exactly s fraction digits, E-notation
//     when the adjusted exponent is below -6) into fixed 48-byte slots, so no length pass / scan is needed: the
//     slots feed the JSON serializers as raw-text columns and CAST AS STRING.
#include "dxa_common.h"

namespace {

typedef unsigned __int128 u128;
constexpr int kSlot = 48;

__device__ __forceinline__ u128 pow10_u128(int k) {
  u128 r = 1;
  for (int i = 0; i < k; ++i) r *= 10;
  return r;
}

__device__ __forceinline__ bool is_ws(uint8_t c) { return c <= 0x20; }

__global__ void dec_from_text_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                     const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                                     int32_t precision, int32_t scale, int32_t trim, int32_t wide,
                                     int64_t* __restrict__ out, uint8_t* __restrict__ ok) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool good = valid == nullptr || valid[i] != 0;
  u128 acc = 0;
  bool neg = false;
  if (good) {
    const uint8_t* s = arena + starts[i];
    int32_t b = 0, e = lens[i];
    if (trim) {
      while (b < e && is_ws(s[b])) ++b;
      while (e > b && is_ws(s[e - 1])) --e;
    }
    int32_t p = b;
    if (p < e && (s[p] == '-' || s[p] == '+')) { neg = s[p] == '-'; ++p; }
    // structure: int digits [p, ie), fraction digits [fs, fe), exponent
    const int32_t is = p;
    while (p < e && s[p] >= '0' && s[p] <= '9') ++p;
    const int32_t ie = p;
    int32_t fs = p, fe = p;
    if (p < e && s[p] == '.') {
      fs = ++p;
      while (p < e && s[p] >= '0' && s[p] <= '9') ++p;
      fe = p;
    }
    int64_t ex = 0;
    if ((ie - is) + (fe - fs) == 0) good = false;
    if (good && p < e && (s[p] | 0x20) == 'e') {
      ++p;
      bool eneg = false;
      if (p < e && (s[p] == '-' || s[p] == '+')) { eneg = s[p] == '-'; ++p; }
      const int32_t es = p;
      while (p < e && s[p] >= '0' && s[p] <= '9') {
        if (ex < 100000) ex = ex * 10 + (s[p] - '0');
        ++p;
      }
      if (p == es) good = false;
      if (eneg) ex = -ex;
    }
    if (p != e) good = false;
    if (good) {
      // digit j (0-based over int then fraction digits) has power (D-1-j) + k in unscaled units
      const int32_t D = (ie - is) + (fe - fs);
      const int64_t k = ex - (fe - fs) + scale;
      const u128 limit = pow10_u128(precision);
      const u128 lim10 = limit / 10;                       // acc ≤ lim10 keeps acc·10 + 9 below 2^128
      int32_t round_digit = 0;
      for (int32_t j = 0; j < D; ++j) {
        const int32_t pos = j < (ie - is) ? is + j : fs + (j - (ie - is));
        const int64_t pw = (int64_t)(D - 1 - j) + k;
        const int32_t d = s[pos] - '0';
        if (pw >= 0) {
          if (acc > lim10) { acc = limit; continue; }      // overflowed: keep scanning for syntax only
          acc = acc * 10 + (u128)d;
        } else if (pw == -1) {
          round_digit = d;
        }
      }
      if (acc != 0 && k > 0) {
        for (int64_t m = 0; m < k; ++m) {
          if (acc > lim10) { acc = limit; break; }
          acc *= 10;
        }
      }
      if (round_digit >= 5) acc += 1;
      if (acc >= limit) good = false;
    }
  }
  u128 v = neg ? (u128)0 - acc : acc;
  if (!good) v = 0;
  if (wide) {
    out[2 * i] = (int64_t)(uint64_t)v;
    out[2 * i + 1] = (int64_t)(uint64_t)(v >> 64);
  } else {
    out[i] = (int64_t)(uint64_t)v;
  }
  ok[i] = good ? 1 : 0;
}

__global__ void dec_to_text_kernel(const int64_t* __restrict__ data, int32_t wide, int32_t scale,
                                   const uint8_t* __restrict__ valid, int64_t n, uint8_t* __restrict__ arena,
                                   int64_t* __restrict__ starts, int32_t* __restrict__ lens) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* o = arena + i * kSlot;
  starts[i] = i * kSlot;
  if (valid != nullptr && !valid[i]) { lens[i] = 0; return; }
  u128 v;
  if (wide) v = ((u128)(uint64_t)data[2 * i + 1] << 64) | (u128)(uint64_t)data[2 * i];
  else v = (u128)(__int128)data[i];
  const bool neg = (__int128)v < 0;
  u128 m = neg ? (u128)0 - v : v;
  char dig[40];
  int nd = 0;
  do {                                                     // at most 39 digits (|v| < 10^38)
    const u128 q = m / 10;
    dig[nd++] = (char)('0' + (int)(m - q * 10));
    m = q;
  } while (m != 0 && nd < 40);
  // dig[] holds the digits least significant first
  int L = 0;
  if (neg) o[L++] = '-';
  const int adjusted = nd - 1 - scale;
  if (adjusted >= -6) {
    if (scale == 0) {
      for (int j = nd - 1; j >= 0; --j) o[L++] = dig[j];
    } else if (nd > scale) {
      for (int j = nd - 1; j >= scale; --j) o[L++] = dig[j];
      o[L++] = '.';
      for (int j = scale - 1; j >= 0; --j) o[L++] = dig[j];
    } else {
      o[L++] = '0';
      o[L++] = '.';
      for (int j = scale - 1; j >= 0; --j) o[L++] = j < nd ? dig[j] : '0';
    }
  } else {
    o[L++] = dig[nd - 1];
    if (nd > 1) {
      o[L++] = '.';
      for (int j = nd - 2; j >= 0; --j) o[L++] = dig[j];
    }
    o[L++] = 'E';
    o[L++] = '-';
    int a = -adjusted;                                     // 7 … 38
    if (a >= 10) o[L++] = (char)('0' + a / 10);
    o[L++] = (char)('0' + a % 10);
  }
  lens[i] = L;
}

}  // namespace

DXA_API int dxa_dec_slot_bytes() { return kSlot; }

DXA_API int dxa_dec_from_text(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                              int64_t n, int32_t precision, int32_t scale, int32_t trim, int32_t wide, int64_t* out,
                              uint8_t* ok, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dec_from_text_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts,
                     lens, valid, n, precision, scale, trim, wide, out, ok);
  return (int)hipGetLastError();
}

DXA_API int dxa_dec_to_text(const int64_t* data, int32_t wide, int32_t scale, const uint8_t* valid, int64_t n,
                            uint8_t* arena, int64_t* starts, int32_t* lens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dec_to_text_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, data, wide, scale,
                     valid, n, arena, starts, lens);
  return (int)hipGetLastError();
}
