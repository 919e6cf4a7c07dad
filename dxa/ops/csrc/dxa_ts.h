// stringToTimestamp (the reference's UDF, UdfInitializer.scala) for one string, shared by the string-function kernel
// (strings.hip) and the JSON parser's timestamp shadow of a string field (json_parse.hip): java.sql.Timestamp.valueOf
// ("yyyy-[m]m-[d]d hh:mm:ss[.f…]"), then "yyyy-MM-dd'T'HH:mm:ss'Z'", then "MM/dd/yyyy HH:mm:ss"; anything else →
// false.  Times are UTC.  Reads only the aligned 8-byte words that overlap [s, s + l) (arenas carry >= 8 B of pad).
#pragma once
#include "dxa_common.h"

namespace dxa {
namespace ts {

__device__ __forceinline__ bool dig(uint8_t c) { return (unsigned)(c - '0') < 10u; }

__device__ inline bool rd(const uint8_t* s, int32_t l, int32_t& i, int minD, int maxD, int& v) {
  v = 0;
  int k = 0;
  while (i < l && k < maxD && dig(s[i])) { v = v * 10 + (s[i] - '0'); ++i; ++k; }
  return k >= minD;
}

}  // namespace ts

__device__ __forceinline__ bool string_to_ts(const uint8_t* s, int32_t l, int64_t& us) {
  using ts::dig;
  using ts::rd;
  bool ok = true;
  int y = 0, mo = 0, d = 0, hh = 0, mi = 0, ss = 0;
  int64_t frac = 0;
  bool fast = false;
  if (ok && l >= 19 && l <= 29) {
    // fixed-width forms ("yyyy-MM-ddTHH:mm:ssZ", "yyyy-MM-dd HH:mm:ss[.f…]") from the aligned 8-B words that
    // overlap the string (never past them), instead of one divergent byte load per character
    const uintptr_t a = reinterpret_cast<uintptr_t>(s);
    const int m = (int)(a & 7);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(a - m);
    uint64_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = (8 * k < m + l) ? q[k] : 0ull;
    uint64_t u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = m ? ((w[k] >> (8 * m)) | (w[k + 1] << (64 - 8 * m))) : w[k];
    auto at = [&](int i) -> int { return (int)((u[i >> 3] >> (8 * (i & 7))) & 0xffu); };
    auto dg = [&](int i) -> int { return at(i) - '0'; };
    bool good = at(4) == '-' && at(7) == '-' && (at(10) == 'T' || at(10) == ' ') && at(13) == ':' &&
                at(16) == ':';
    const int pos[14] = {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18};
#pragma unroll
    for (int k = 0; k < 14; ++k) good = good && (unsigned)dg(pos[k]) < 10u;
    if (good) {
      const bool iso = at(10) == 'T';
      if (iso) {
        good = l == 20 && at(19) == 'Z';
      } else if (l > 19) {
        good = l >= 21 && at(19) == '.';
        int64_t scale = 100000;
#pragma unroll
        for (int i = 20; i < 29; ++i) {
          if (i < l) {
            const int c = dg(i);
            good = good && (unsigned)c < 10u;
            frac += c * scale;
            scale /= 10;
          }
        }
      }
    }
    if (good) {
      y = dg(0) * 1000 + dg(1) * 100 + dg(2) * 10 + dg(3);
      mo = dg(5) * 10 + dg(6);
      d = dg(8) * 10 + dg(9);
      hh = dg(11) * 10 + dg(12);
      mi = dg(14) * 10 + dg(15);
      ss = dg(17) * 10 + dg(18);
      fast = true;
      ok = !(mo < 1 || mo > 12 || d < 1 || d > 31 || hh > 23 || mi > 59 || ss > 59);
    } else {
      frac = 0;
    }
  }
  if (ok && !fast) {
    ok = false;
    int32_t i = 0;
    // form A / B: yyyy-M-d( |T)HH:mm:ss[.f][Z]
    if (rd(s, l, i, 4, 4, y) && i < l && s[i] == '-') {
      ++i;
      if (rd(s, l, i, 1, 2, mo) && i < l && s[i] == '-') {
        ++i;
        if (rd(s, l, i, 1, 2, d) && i < l && (s[i] == ' ' || s[i] == 'T')) {
          const bool iso = s[i] == 'T';
          ++i;
          if (rd(s, l, i, 1, 2, hh) && i < l && s[i] == ':' && (++i, rd(s, l, i, 1, 2, mi)) && i < l &&
              s[i] == ':' && (++i, rd(s, l, i, 1, 2, ss))) {
            if (!iso && i < l && s[i] == '.') {
              ++i;
              int64_t scale = 100000;
              int nd = 0;
              while (i < l && dig(s[i])) { if (scale) { frac += (s[i] - '0') * scale; scale /= 10; } ++i; ++nd; }
              ok = nd > 0 && i == l;
            } else if (iso) {
              ok = (i + 1 == l && s[i] == 'Z');
            } else {
              ok = i == l;
            }
          }
        }
      }
    }
    if (!ok) {
      // form C: MM/dd/yyyy HH:mm:ss
      i = 0;
      frac = 0;
      if (rd(s, l, i, 1, 2, mo) && i < l && s[i] == '/' && (++i, rd(s, l, i, 1, 2, d)) && i < l && s[i] == '/' &&
          (++i, rd(s, l, i, 4, 4, y)) && i < l && s[i] == ' ' && (++i, rd(s, l, i, 1, 2, hh)) && i < l &&
          s[i] == ':' && (++i, rd(s, l, i, 1, 2, mi)) && i < l && s[i] == ':' && (++i, rd(s, l, i, 1, 2, ss)))
        ok = i == l;
    }
    if (ok && (mo < 1 || mo > 12 || d < 1 || d > 31 || hh > 23 || mi > 59 || ss > 59)) ok = false;
  }
  if (!ok) return false;
  const int64_t days = dxa::days_from_civil(y, (unsigned)mo, (unsigned)d);
  us = (days * 86400 + hh * 3600 + mi * 60 + ss) * 1000000ll + frac;
  return true;
}

}  // namespace dxa
