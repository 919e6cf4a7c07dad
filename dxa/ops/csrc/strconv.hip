// Device number ↔ text and codec built-ins (user SQL runs in Spark 2.4 codegen on the executors,
// CommonProcessorFactory.scala:257-275): format_number, conv / bin, soundex, unhex, unbase64, split_part.
//
// Shapes (one lane per row):
//   * fixed-slot outputs (format_number ≤ 64 bytes, conv / bin ≤ 66, soundex 4) go straight into [n × slot] arenas:
//     no length pass, no scan, no host read;
//   * unhex / unbase64 outputs are at most the input length: a length pass, a scan, a write pass;
//   * split_part is a view (start, length) into the input arena.
// Decoded bytes that are not UTF-8 become U+FFFD per maximal ill-formed subpart (utf8_clean, Python's
// errors="replace"), as the host path renders them.  Rows a kernel does not reproduce exactly flag `bad`
// (format_number beyond 10^18 or NaN / ±Inf, soundex inputs Spark returns unchanged); the caller then evaluates
// the column on the host (the CPU evaluator, the differential tests' oracle).
#include "dxa_common.h"
#include "dxa_ryu.h"

namespace {

__constant__ uint64_t c_ryu_inv[2 * DXA_RYU_INV_TABLE_SIZE] = DXA_RYU_POW5_INV_SPLIT_INIT;
__constant__ uint64_t c_ryu_pos[2 * DXA_RYU_TABLE_SIZE] = DXA_RYU_POW5_SPLIT_INIT;

constexpr int kFmtSlot = 64;
constexpr int kConvSlot = 66;

__device__ __forceinline__ uint64_t pow10u(int k) {
  uint64_t r = 1;
  for (int i = 0; i < k; ++i) r *= 10;
  return r;
}

// decimal digits of v (most significant first) into out; returns the count (v == 0 → "0")
__device__ __forceinline__ int u64_digits(uint64_t v, char* out) {
  char tmp[20];
  int n = 0;
  do {
    tmp[n++] = (char)('0' + (int)(v % 10));
    v /= 10;
  } while (v);
  for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
  return n;
}

// format_number(x, d): java.text.DecimalFormat("#,##0.000…") with RoundingMode.HALF_EVEN over the value's shortest
// decimal digits.  q = round(D · 10^(e + d)) as a digit string, then "int,part.frac".
__device__ bool format_one(bool neg, uint64_t D, int32_t e, int32_t d, uint8_t* o, int32_t& len) {
  char S[20];
  const int L = u64_digits(D, S);
  char Q[64];
  int ql = 0;
  const int32_t t = e + d;
  if (t >= 0) {
    if (L + t > 60) return false;
    for (int i = 0; i < L; ++i) Q[ql++] = S[i];
    for (int i = 0; i < t; ++i) Q[ql++] = '0';
  } else {
    const int k = -t;
    uint64_t q;
    if (k > L) {
      q = 0;
    } else if (k == L) {
      const uint64_t half = 5 * pow10u(L - 1);
      q = (D > half) ? 1 : 0;                              // == half: round to the even 0
    } else {
      const uint64_t p = pow10u(k);
      q = D / p;
      const uint64_t r = D - q * p, half = p / 2;
      if (r > half || (r == half && (q & 1))) ++q;
    }
    ql = u64_digits(q, Q);
  }
  // at least d + 1 digits: leading zeros
  if (ql < d + 1) {
    const int pad = d + 1 - ql;
    for (int i = ql - 1; i >= 0; --i) Q[i + pad] = Q[i];
    for (int i = 0; i < pad; ++i) Q[i] = '0';
    ql += pad;
  }
  const int il = ql - d;                                   // integer digits
  if (il > 18) return false;
  int p = 0;
  if (neg) o[p++] = '-';
  for (int i = 0; i < il; ++i) {
    o[p++] = (uint8_t)Q[i];
    const int rest = il - 1 - i;
    if (rest > 0 && rest % 3 == 0) o[p++] = ',';
  }
  if (d > 0) {
    o[p++] = '.';
    for (int i = il; i < ql; ++i) o[p++] = (uint8_t)Q[i];
  }
  len = p;
  return true;
}

__global__ void format_number_kernel(const void* __restrict__ data, int32_t is_f64, const uint8_t* __restrict__ valid,
                                     int64_t n, int32_t d, uint8_t* __restrict__ arena, int64_t* __restrict__ starts,
                                     int32_t* __restrict__ lens, int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t* o = arena + i * kFmtSlot;
    starts[i] = i * kFmtSlot;
    int32_t len = 0;
    if (valid == nullptr || valid[i]) {
      bool neg, ok = true;
      uint64_t D;
      int32_t e;
      if (is_f64) {
        const double v = ((const double*)data)[i];
        neg = __double_as_longlong(v) < 0;
        if (!(v == v) || v == __builtin_inf() || v == -__builtin_inf()) {
          ok = false;
          D = 0;
          e = 0;
        } else if (v == 0.0) {
          D = 0;
          e = 0;
        } else {
          dxa::ryu::d2d(neg ? -v : v, D, e, c_ryu_inv, c_ryu_pos);
        }
      } else {
        const int64_t v = ((const int64_t*)data)[i];
        neg = v < 0;
        D = neg ? 0ull - (uint64_t)v : (uint64_t)v;
        e = 0;
      }
      if (!ok || !format_one(neg, D, e, d, o, len)) {
        atomicAdd(bad, 1);
        len = 0;
      }
    }
    lens[i] = len;
  }
}

__device__ __forceinline__ int digit_of(uint8_t c, int radix) {       // java.lang.Character.digit on one byte
  int v;
  if (c >= '0' && c <= '9') v = c - '0';
  else if (c >= 'a' && c <= 'z') v = c - 'a' + 10;
  else if (c >= 'A' && c <= 'Z') v = c - 'A' + 10;
  else return -1;
  return v < radix ? v : -1;
}

// unsigned 64-bit → text in base b (upper-case digits), Hive/Spark NumberConverter.decode + byte2char
__device__ __forceinline__ int u64_to_base(uint64_t v, int b, bool minus, uint8_t* o) {
  char tmp[64];
  int n = 0;
  do {
    const int r = (int)(v % (uint64_t)b);
    tmp[n++] = (char)(r < 10 ? '0' + r : 'A' + r - 10);
    v /= (uint64_t)b;
  } while (v);
  int p = 0;
  if (minus) o[p++] = '-';
  for (int i = n - 1; i >= 0; --i) o[p++] = (uint8_t)tmp[i];
  return p;
}

// conv(num, from, to): Spark 2.4 NumberConverter.convert over the space-trimmed bytes
__global__ void conv_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                            const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                            int32_t from, int32_t to, uint8_t* __restrict__ out, int64_t* __restrict__ ostarts,
                            int32_t* __restrict__ olens, uint8_t* __restrict__ ovalid) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + i * kConvSlot;
    ostarts[i] = i * kConvSlot;
    olens[i] = 0;
    ovalid[i] = 0;
    if (valid != nullptr && !valid[i]) continue;
    const uint8_t* s = arena + starts[i];
    int32_t b = 0, e = lens[i];
    while (b < e && s[b] == ' ') ++b;
    while (e > b && s[e - 1] == ' ') --e;
    if (e == b) continue;                                  // empty → NULL
    bool neg = s[b] == '-';
    const int32_t first = b + (neg ? 1 : 0);
    if (e - first > 64) continue;                          // the reference's 64-byte buffer overflows: NULL here
    // encode: stop at the first non-digit; saturate to all ones on unsigned overflow
    uint64_t v = 0;
    const uint64_t bound = (~0ull - (uint64_t)from) / (uint64_t)from;
    for (int32_t k = first; k < e; ++k) {
      const int dg = digit_of(s[k], from);
      if (dg < 0) break;
      if (v >= bound && (~0ull - (uint64_t)dg) / (uint64_t)from < v) { v = ~0ull; break; }
      v = v * (uint64_t)from + (uint64_t)dg;
    }
    if (neg && to > 0) v = ((int64_t)v < 0) ? ~0ull : 0ull - v;
    if (to < 0 && (int64_t)v < 0) { v = 0ull - v; neg = true; }
    olens[i] = u64_to_base(v, to < 0 ? -to : to, neg && to < 0, o);
    ovalid[i] = 1;
  }
}

__global__ void bin_kernel(const int64_t* __restrict__ data, int64_t n, uint8_t* __restrict__ out,
                           int64_t* __restrict__ ostarts, int32_t* __restrict__ olens) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    ostarts[i] = i * kConvSlot;
    olens[i] = u64_to_base((uint64_t)data[i], 2, false, out + i * kConvSlot);
  }
}

// soundex (UTF8String.soundex): rows whose first byte is not an ASCII letter are returned unchanged by Spark — they
// set `bad` (the caller keeps such columns on the host path)
__global__ void soundex_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                               const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                               uint8_t* __restrict__ out, int64_t* __restrict__ ostarts, int32_t* __restrict__ olens,
                               int32_t* __restrict__ bad) {
  // US English mapping A..Z: '7' marks H and W (skipped without resetting the last code)
  const char* map = "01230127022455012623017202";
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + i * 4;
    ostarts[i] = i * 4;
    olens[i] = 0;
    if (valid != nullptr && !valid[i]) continue;
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    if (l == 0) continue;                                  // "" → ""
    uint8_t c = s[0];
    if (c >= 'a' && c <= 'z') c -= 32;
    if (c < 'A' || c > 'Z') { atomicAdd(bad, 1); continue; }
    uint8_t sx[4] = {c, '0', '0', '0'};
    int sxi = 1;
    char last = map[c - 'A'];
    for (int32_t k = 1; k < l && sxi < 4; ++k) {
      uint8_t b = s[k];
      if (b >= 'a' && b <= 'z') b -= 32;
      if (b < 'A' || b > 'Z') { last = '0'; continue; }
      const char code = map[b - 'A'];
      if (code == '7') continue;
      if (code != '0' && code != last) sx[sxi++] = (uint8_t)code;
      last = code;
    }
    for (int k = 0; k < 4; ++k) o[k] = sx[k];
    olens[i] = 4;
  }
}

__device__ __forceinline__ int hexval(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// commons-codec Base64 decode table: standard and URL-safe alphabets; -1 = ignored byte
__device__ __forceinline__ int b64val(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+' || c == '-') return 62;
  if (c == '/' || c == '_') return 63;
  return -1;
}

// mode 0 = unhex (Hex.unhex: an odd length pads a leading '0'; any non-hex byte → NULL), 1 = unbase64 (lenient
// commons-codec decode: bytes outside the alphabet are skipped, '=' ends the data, a trailing 2 / 3-symbol group
// yields 1 / 2 bytes).  Pass 1 (dst == nullptr): output length per row; pass 2: write at off[i].
__global__ void decode_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                              const int32_t* __restrict__ lens, const uint8_t* __restrict__ valid, int64_t n,
                              int32_t mode, const int64_t* __restrict__ off, uint8_t* __restrict__ dst,
                              int64_t* __restrict__ out_len, uint8_t* __restrict__ ovalid, int32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool write = dst != nullptr;
    if (valid != nullptr && !valid[i]) {
      if (!write) { out_len[i] = 0; ovalid[i] = 0; }
      continue;
    }
    // a row the length pass rejected owns no output bytes: decoding its valid prefix would write into the next
    // row's slot
    if (write && !ovalid[i]) continue;
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* o = write ? dst + off[i] : nullptr;
    int64_t p = 0;
    bool ok = true, ascii = true;
    if (mode == 0) {
      int32_t k = 0;
      if (l & 1) {
        const int v = hexval(s[0]);
        if (v < 0) ok = false;
        else {
          if (write) o[p] = (uint8_t)v;
          ++p;
        }
        k = 1;
      }
      for (; ok && k + 1 < l; k += 2) {
        const int a = hexval(s[k]), b = hexval(s[k + 1]);
        if (a < 0 || b < 0) { ok = false; break; }
        const uint8_t byte = (uint8_t)((a << 4) | b);
        ascii &= byte < 0x80;
        if (write) o[p] = byte;
        ++p;
      }
    } else {
      uint32_t acc = 0;
      int m = 0;
      for (int32_t k = 0; k < l; ++k) {
        const uint8_t c = s[k];
        if (c == '=') break;
        const int v = b64val(c);
        if (v < 0) continue;
        acc = (acc << 6) | (uint32_t)v;
        if (++m == 4) {
          const uint8_t b0 = (uint8_t)(acc >> 16), b1 = (uint8_t)(acc >> 8), b2 = (uint8_t)acc;
          ascii &= (b0 | b1 | b2) < 0x80;
          if (write) { o[p] = b0; o[p + 1] = b1; o[p + 2] = b2; }
          p += 3;
          m = 0;
          acc = 0;
        }
      }
      if (m >= 2) {
        const uint8_t b0 = (uint8_t)(acc >> (m == 2 ? 4 : 10));
        ascii &= b0 < 0x80;
        if (write) o[p] = b0;
        ++p;
        if (m == 3) {
          const uint8_t b1 = (uint8_t)(acc >> 2);
          ascii &= b1 < 0x80;
          if (write) o[p] = b1;
          ++p;
        }
      }
    }
    if (!write) {
      out_len[i] = ok ? p : 0;
      ovalid[i] = ok ? 1 : 0;
      (void)ascii;
    }
  }
}

// split_part(s, delim, k) (Spark 3.3 semantics): k > 0 counts fields from the start, k < 0 from the end; a field
// index out of range → ""; an empty delimiter makes the whole string the only field
__global__ void split_part_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, int64_t n, const uint8_t* __restrict__ dl,
                                  int32_t dn, int64_t k, int64_t* __restrict__ out_start,
                                  int32_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    int64_t st = starts[i];
    int32_t ln = 0;
    if (dn == 0) {
      if (k == 1 || k == -1) ln = l;
    } else if (k > 0) {
      int64_t field = 1;
      int32_t fs = 0, q = 0;
      bool found = false;
      while (q + dn <= l) {
        bool m = true;
        for (int32_t z = 0; z < dn && m; ++z) m = s[q + z] == dl[z];
        if (m) {
          if (field == k) { st = starts[i] + fs; ln = q - fs; found = true; break; }
          ++field;
          q += dn;
          fs = q;
        } else {
          ++q;
        }
      }
      if (!found && field == k) { st = starts[i] + fs; ln = l - fs; }
    } else {
      int64_t field = 1;
      int32_t fe = l, q = l - dn;
      bool found = false;
      while (q >= 0) {
        bool m = true;
        for (int32_t z = 0; z < dn && m; ++z) m = s[q + z] == dl[z];
        if (m) {
          if (field == -k) { st = starts[i] + q + dn; ln = fe - q - dn; found = true; break; }
          ++field;
          fe = q;
          q -= dn;
        } else {
          --q;
        }
      }
      if (!found && field == -k) { st = starts[i]; ln = fe; }
    }
    out_start[i] = st;
    out_len[i] = ln;
  }
}

// UTF-8 validation with Python's errors="replace" (the Unicode "maximal subpart" policy): a well-formed sequence is
// copied, every maximal ill-formed subpart becomes U+FFFD (EF BF BD).  Returns the byte length of the clean text.
__device__ int64_t utf8_clean(const uint8_t* s, int32_t l, uint8_t* o, bool& changed) {
  int64_t p = 0;
  int32_t k = 0;
  while (k < l) {
    const uint8_t c = s[k];
    if (c < 0x80) {
      if (o) o[p] = c;
      ++p;
      ++k;
      continue;
    }
    int need;
    uint8_t lo = 0x80, hi = 0xBF;                          // bounds of the first continuation byte
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else need = -1;
    int got = 0;
    if (need > 0) {
      while (got < need && k + 1 + got < l) {
        const uint8_t b = s[k + 1 + got];
        const uint8_t blo = got == 0 ? lo : 0x80, bhi = got == 0 ? hi : 0xBF;
        if (b < blo || b > bhi) break;
        ++got;
      }
    }
    if (need > 0 && got == need) {
      for (int z = 0; z <= need; ++z) {
        if (o) o[p] = s[k + z];
        ++p;
      }
      k += need + 1;
    } else {
      if (o) { o[p] = 0xEF; o[p + 1] = 0xBF; o[p + 2] = 0xBD; }
      p += 3;
      k += 1 + got;
      changed = true;
    }
  }
  return p;
}

// pass 1 (dst == nullptr): clean lengths + the count of rows that change; pass 2: write at off[i]
__global__ void utf8_clean_kernel(const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                  const int32_t* __restrict__ lens, int64_t n, const int64_t* __restrict__ off,
                                  uint8_t* __restrict__ dst, int64_t* __restrict__ out_len,
                                  int32_t* __restrict__ changed_rows) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    bool changed = false;
    const int64_t L = utf8_clean(arena + starts[i], lens[i], dst ? dst + off[i] : nullptr, changed);
    if (!dst) {
      out_len[i] = L;
      if (changed) atomicAdd(changed_rows, 1);
    }
  }
}

}  // namespace

DXA_API int dxa_utf8_clean(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           const int64_t* off, uint8_t* dst, int64_t* out_len, int32_t* changed_rows, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(utf8_clean_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, off, dst, out_len, changed_rows);
  return (int)hipGetLastError();
}

DXA_API int dxa_fmt_slot_bytes() { return kFmtSlot; }
DXA_API int dxa_conv_slot_bytes() { return kConvSlot; }

DXA_API int dxa_format_number(const void* data, int32_t is_f64, const uint8_t* valid, int64_t n, int32_t d,
                              uint8_t* arena, int64_t* starts, int32_t* lens, int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(format_number_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, data, is_f64,
                     valid, n, d, arena, starts, lens, bad);
  return (int)hipGetLastError();
}

DXA_API int dxa_conv(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid, int64_t n,
                     int32_t from, int32_t to, uint8_t* out, int64_t* ostarts, int32_t* olens, uint8_t* ovalid,
                     void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(conv_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens, valid,
                     n, from, to, out, ostarts, olens, ovalid);
  return (int)hipGetLastError();
}

DXA_API int dxa_bin(const int64_t* data, int64_t n, uint8_t* out, int64_t* ostarts, int32_t* olens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(bin_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, data, n, out, ostarts,
                     olens);
  return (int)hipGetLastError();
}

DXA_API int dxa_soundex(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                        int64_t n, uint8_t* out, int64_t* ostarts, int32_t* olens, int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(soundex_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, n, out, ostarts, olens, bad);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_decode(const uint8_t* arena, const int64_t* starts, const int32_t* lens, const uint8_t* valid,
                           int64_t n, int32_t mode, const int64_t* off, uint8_t* dst, int64_t* out_len,
                           uint8_t* ovalid, int32_t* bad, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(decode_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     valid, n, mode, off, dst, out_len, ovalid, bad);
  return (int)hipGetLastError();
}

DXA_API int dxa_split_part(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n,
                           const uint8_t* dl, int32_t dn, int64_t k, int64_t* out_start, int32_t* out_len, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(split_part_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, dl, dn, k, out_start, out_len);
  return (int)hipGetLastError();
}
