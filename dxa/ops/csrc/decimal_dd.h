// Decimal → double with one final rounding, shared by the JSON parser and CAST(string AS DOUBLE).
//
// The digits arrive as two 19-digit halves: value = head × 10^e10 + tail × 10^(e10 − nt), where head holds the
// first 19 significant digits and tail the next nt (≤ 19).  Keeping the second half matters: truncating at 19
// digits moves the value by up to 1e-19 relative, which flips the rounding of about one long-mantissa number in a
// thousand; with 38 digits the residual error is below the double-double product's own (≈2^-104).
#pragma once
#include <stdint.h>

#include "pow10_dd.h"

// head ≠ 0 and DXA_POW10_DD_MIN ≤ e10 ≤ DXA_POW10_DD_MAX (the caller handles 0 / overflow / underflow and its
// exact small-exponent fast paths).
__device__ __forceinline__ double dxa_decimal_to_double(uint64_t head, int e10, uint64_t tail, int nt) {
#pragma clang fp contract(off)
  // head (exact as hi + lo) × 10^e10 (double-double).  No contraction: fusing h = mh*ph into a later add would
  // count the product's rounding error twice
  const bool wide = head >= (1ull << 53);
  const double mh = (double)(wide ? (head & ~0x7FFull) : head), ml = wide ? (double)(head & 0x7FFull) : 0.0;
  const double ph = kPow10dd[e10 - DXA_POW10_DD_MIN][0], pl = kPow10dd[e10 - DXA_POW10_DD_MIN][1];
  const double h = mh * ph;
  if (__builtin_isinf(h)) return h;                       // overflow (inf − inf in the error term would be NaN)
  const double err = __builtin_fma(mh, ph, -h) + (mh * pl + ml * ph);
  double b = 0.0;                                         // tail term: ≤ 1e-19 of h, plain double precision is enough
  const int e2 = e10 - nt;
  if (tail != 0 && e2 >= DXA_POW10_DD_MIN) {
    b = (double)tail * kPow10dd[e2 - DXA_POW10_DD_MIN][0];
    if (e2 < DXA_POW10_DD_SCALED_BELOW && e10 >= DXA_POW10_DD_SCALED_BELOW)
      b = __builtin_ldexp(b, -DXA_POW10_DD_SCALE);        // tail's entry is scaled, head's is not
  }
  const double s = h + b;                                 // two-sum(h, b)
  const double bb = s - h;
  const double es = (h - (s - bb)) + (b - bb);
  double d = s + (es + err);
  if (e10 < DXA_POW10_DD_SCALED_BELOW) d = __builtin_ldexp(d, -DXA_POW10_DD_SCALE);   // exact power-of-2 scale
  return d;
}
