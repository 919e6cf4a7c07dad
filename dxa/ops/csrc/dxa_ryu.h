// Shortest round-trip double → decimal (Ryu, Ulf Adams PLDI 2018) and Java Double.toString text, as
// __host__ __device__ code: the GPU JSON serializer renders doubles on the device, and the same code is called on
// the CPU by the tests that check it against the host formatter.  Tables are passed in (device: __constant__ copy,
// host: static copy) so one implementation serves both sides.
#pragma once
#include <cstdint>

#include "ryu_tables.h"

namespace dxa {
namespace ryu {

__host__ __device__ inline uint32_t pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1; }
__host__ __device__ inline uint32_t log10pow2(int32_t e) { return ((uint32_t)e * 78913u) >> 18; }
__host__ __device__ inline uint32_t log10pow5(int32_t e) { return ((uint32_t)e * 732923u) >> 20; }

__host__ __device__ inline uint32_t pow5factor(uint64_t v) {
  uint32_t c = 0;
  for (;;) {
    const uint64_t q = v / 5;
    if (v - 5 * q != 0) break;
    v = q;
    ++c;
  }
  return c;
}
__host__ __device__ inline bool multiple_of_pow5(uint64_t v, uint32_t p) { return pow5factor(v) >= p; }
__host__ __device__ inline bool multiple_of_pow2(uint64_t v, uint32_t p) { return (v & ((1ull << p) - 1)) == 0; }

// ((m * mul) >> j) with mul a 128-bit {lo, hi} table entry, j >= 64
__host__ __device__ inline uint64_t mul_shift(uint64_t m, const uint64_t* mul, int32_t j) {
  const unsigned __int128 b0 = (unsigned __int128)m * mul[0];
  const unsigned __int128 b2 = (unsigned __int128)m * mul[1];
  return (uint64_t)(((b0 >> 64) + b2) >> (j - 64));
}

__host__ __device__ inline uint32_t decimal_len(uint64_t v) {
  uint32_t n = 1;
  uint64_t p = 10;
  while (n < 17 && v >= p) { ++n; p *= 10; }
  return n;
}

// v finite and non-zero → shortest digits (as an integer) and decimal exponent: |v| = digits * 10^exp
__host__ __device__ inline void d2d(double v, uint64_t& digits, int32_t& exp10, const uint64_t* inv_tab,
                                    const uint64_t* tab) {
  uint64_t bits;
  __builtin_memcpy(&bits, &v, 8);
  const uint64_t mant = bits & ((1ull << 52) - 1);
  const uint32_t ex = (uint32_t)((bits >> 52) & 0x7ff);
  int32_t e2;
  uint64_t m2;
  if (ex == 0) {
    e2 = 1 - 1023 - 52 - 2;
    m2 = mant;
  } else {
    e2 = (int32_t)ex - 1023 - 52 - 2;
    m2 = (1ull << 52) | mant;
  }
  const bool even = (m2 & 1) == 0;
  const bool accept = even;
  const uint64_t mv = 4 * m2;
  const uint32_t mm_shift = (mant != 0 || ex <= 1) ? 1 : 0;
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;
  if (e2 >= 0) {
    const uint32_t q = log10pow2(e2) - (e2 > 3);
    e10 = (int32_t)q;
    const int32_t k = DXA_RYU_POW5_INV_BITCOUNT + (int32_t)pow5bits((int32_t)q) - 1;
    const int32_t i = -e2 + (int32_t)q + k;
    const uint64_t* mul = inv_tab + 2 * q;
    vr = mul_shift(4 * m2, mul, i);
    vp = mul_shift(4 * m2 + 2, mul, i);
    vm = mul_shift(4 * m2 - 1 - mm_shift, mul, i);
    if (q <= 21) {
      const uint32_t mv_mod5 = (uint32_t)(mv % 5);
      if (mv_mod5 == 0) vr_tz = multiple_of_pow5(mv, q);
      else if (accept) vm_tz = multiple_of_pow5(mv - 1 - mm_shift, q);
      else vp -= multiple_of_pow5(mv + 2, q);
    }
  } else {
    const uint32_t q = log10pow5(-e2) - (-e2 > 1);
    e10 = (int32_t)q + e2;
    const int32_t i = -e2 - (int32_t)q;
    const int32_t k = (int32_t)pow5bits(i) - DXA_RYU_POW5_BITCOUNT;
    const int32_t j = (int32_t)q - k;
    const uint64_t* mul = tab + 2 * i;
    vr = mul_shift(4 * m2, mul, j);
    vp = mul_shift(4 * m2 + 2, mul, j);
    vm = mul_shift(4 * m2 - 1 - mm_shift, mul, j);
    if (q <= 1) {
      vr_tz = true;
      if (accept) vm_tz = mm_shift == 1;
      else --vp;
    } else if (q < 63) {
      vr_tz = multiple_of_pow2(mv, q);
    }
  }
  int32_t removed = 0;
  uint8_t last = 0;
  uint64_t out;
  if (vm_tz || vr_tz) {
    for (;;) {
      const uint64_t vpd = vp / 10, vmd = vm / 10;
      if (vpd <= vmd) break;
      const uint32_t vm_mod = (uint32_t)(vm - 10 * vmd);
      const uint64_t vrd = vr / 10;
      const uint32_t vr_mod = (uint32_t)(vr - 10 * vrd);
      vm_tz &= vm_mod == 0;
      vr_tz &= last == 0;
      last = (uint8_t)vr_mod;
      vr = vrd; vp = vpd; vm = vmd;
      ++removed;
    }
    if (vm_tz) {
      for (;;) {
        const uint64_t vmd = vm / 10;
        const uint32_t vm_mod = (uint32_t)(vm - 10 * vmd);
        if (vm_mod != 0) break;
        const uint64_t vpd = vp / 10, vrd = vr / 10;
        const uint32_t vr_mod = (uint32_t)(vr - 10 * vrd);
        vr_tz &= last == 0;
        last = (uint8_t)vr_mod;
        vr = vrd; vp = vpd; vm = vmd;
        ++removed;
      }
    }
    if (vr_tz && last == 5 && vr % 2 == 0) last = 4;     // round half to even
    out = vr + ((vr == vm && (!accept || !vm_tz)) || last >= 5);
  } else {
    bool round_up = false;
    for (;;) {
      const uint64_t vpd = vp / 10, vmd = vm / 10;
      if (vpd <= vmd) break;
      const uint64_t vrd = vr / 10;
      const uint32_t vr_mod = (uint32_t)(vr - 10 * vrd);
      round_up = vr_mod >= 5;
      vr = vrd; vp = vpd; vm = vmd;
      ++removed;
    }
    out = vr + (vr == vm || round_up);
  }
  digits = out;
  exp10 = e10 + removed;
}

// Java Double.toString text (JDK 19+ shortest digits): NaN / Infinity / -0.0; plain for 1e-3 <= |v| < 1e7
// ("123.45", "100.0", "0.00123"), otherwise "d.dddE±x" ("1.0E7", "1.234E-5").  Writes at most 26 chars when out is
// non-null; returns the length.
__host__ __device__ inline int java_double(double v, char* out, const uint64_t* inv_tab, const uint64_t* tab) {
  char buf[32];
  char* o = out ? out : buf;
  int n = 0;
  if (v != v) { const char* s = "NaN"; for (int i = 0; i < 3; ++i) o[n++] = s[i]; return n; }
  uint64_t bits;
  __builtin_memcpy(&bits, &v, 8);
  const bool neg = (bits >> 63) != 0;
  if ((bits & 0x7fffffffffffffffull) == 0x7ff0000000000000ull) {
    const char* s = "Infinity";
    if (neg) o[n++] = '-';
    for (int i = 0; i < 8; ++i) o[n++] = s[i];
    return n;
  }
  if ((bits & 0x7fffffffffffffffull) == 0) {
    if (neg) o[n++] = '-';
    o[n++] = '0'; o[n++] = '.'; o[n++] = '0';
    return n;
  }
  uint64_t d;
  int32_t e;
  d2d(v, d, e, inv_tab, tab);
  char dig[20];
  const int len = (int)decimal_len(d);
  for (int i = len - 1; i >= 0; --i) { dig[i] = (char)('0' + d % 10); d /= 10; }
  const int sci = e + len - 1;                  // value = 0.d1d2.. * 10^(sci+1)
  if (neg) o[n++] = '-';
  if (sci >= -3 && sci < 7) {
    const int point = sci + 1;                  // digits before the decimal point
    if (point <= 0) {
      o[n++] = '0'; o[n++] = '.';
      for (int i = 0; i < -point; ++i) o[n++] = '0';
      for (int i = 0; i < len; ++i) o[n++] = dig[i];
    } else if (point >= len) {
      for (int i = 0; i < len; ++i) o[n++] = dig[i];
      for (int i = len; i < point; ++i) o[n++] = '0';
      o[n++] = '.'; o[n++] = '0';
    } else {
      for (int i = 0; i < point; ++i) o[n++] = dig[i];
      o[n++] = '.';
      for (int i = point; i < len; ++i) o[n++] = dig[i];
    }
  } else {
    o[n++] = dig[0];
    o[n++] = '.';
    if (len > 1) { for (int i = 1; i < len; ++i) o[n++] = dig[i]; } else o[n++] = '0';
    o[n++] = 'E';
    int x = sci;
    if (x < 0) { o[n++] = '-'; x = -x; }
    char xb[4];
    int xn = 0;
    do { xb[xn++] = (char)('0' + x % 10); x /= 10; } while (x);
    while (xn) o[n++] = xb[--xn];
  }
  return n;
}

}  // namespace ryu
}  // namespace dxa
