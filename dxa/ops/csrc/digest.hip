// Per-row digests and encodings of string columns, for the SQL functions md5 / sha1 / sha2(…, 0|224|256) / crc32 /
// hex / base64 (Spark: Md5, Sha1, Sha2, Crc32, Hex, Base64 over the UTF-8 bytes).  One lane per row: the message
// blocks are assembled from the row's bytes on the fly (padding and the bit length appended in the last block), so
// nothing is staged.  Digests come out as lower-case hex in fixed-width slots.
#include "dxa_common.h"
#include "digest_tables.h"

namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

// byte k of the padded message (length l bytes, nb blocks): data, 0x80, zeros, then the 64-bit bit length —
// big-endian for SHA, little-endian for MD5
template <bool kBigEndianLen>
__device__ __forceinline__ uint32_t msg_byte(const uint8_t* s, int32_t l, int64_t k, int64_t total) {
  if (k < l) return s[k];
  if (k == l) return 0x80;
  const int64_t lk = k - (total - 8);
  if (lk < 0) return 0;
  const uint64_t bits = (uint64_t)l * 8;
  return kBigEndianLen ? (uint32_t)(bits >> (8 * (7 - lk))) & 0xff : (uint32_t)(bits >> (8 * lk)) & 0xff;
}

__device__ __forceinline__ void put_hex(uint8_t* o, uint32_t byte) {
  const char* d = "0123456789abcdef";
  o[0] = d[byte >> 4];
  o[1] = d[byte & 15];
}

__device__ void md5_row(const uint8_t* s, int32_t l, uint8_t* o) {
  const int64_t total = ((int64_t)l + 8) / 64 * 64 + 64;
  uint32_t h0 = 0x67452301u, h1 = 0xefcdab89u, h2 = 0x98badcfeu, h3 = 0x10325476u;
  constexpr int kR[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
  for (int64_t b = 0; b < total; b += 64) {
    uint32_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint32_t v = 0;
      for (int q = 0; q < 4; ++q) v |= msg_byte<false>(s, l, b + 4 * j + q, total) << (8 * q);
      w[j] = v;
    }
    uint32_t a = h0, bb = h1, c = h2, d = h3;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (bb & c) | (~bb & d); g = i; }
      else if (i < 32) { f = (d & bb) | (~d & c); g = (5 * i + 1) & 15; }
      else if (i < 48) { f = bb ^ c ^ d; g = (3 * i + 5) & 15; }
      else { f = c ^ (bb | ~d); g = (7 * i) & 15; }
      const uint32_t t = d;
      d = c;
      c = bb;
      bb = bb + rotl(a + f + kMd5K[i] + w[g], kR[(i >> 4) * 4 + (i & 3)]);
      a = t;
    }
    h0 += a; h1 += bb; h2 += c; h3 += d;
  }
  const uint32_t hs[4] = {h0, h1, h2, h3};
  for (int i = 0; i < 16; ++i) put_hex(o + 2 * i, (hs[i >> 2] >> (8 * (i & 3))) & 0xff);
}

__device__ void sha1_row(const uint8_t* s, int32_t l, uint8_t* o) {
  const int64_t total = ((int64_t)l + 8) / 64 * 64 + 64;
  uint32_t h[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
  for (int64_t b = 0; b < total; b += 64) {
    uint32_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint32_t v = 0;
      for (int q = 0; q < 4; ++q) v = (v << 8) | msg_byte<true>(s, l, b + 4 * j + q, total);
      w[j] = v;
    }
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int i = 0; i < 80; ++i) {
      uint32_t wi;
      if (i < 16) wi = w[i];
      else { wi = rotl(w[(i - 3) & 15] ^ w[(i - 8) & 15] ^ w[(i - 14) & 15] ^ w[i & 15], 1); w[i & 15] = wi; }
      uint32_t f, k;
      if (i < 20) { f = (bb & c) | (~bb & d); k = 0x5a827999u; }
      else if (i < 40) { f = bb ^ c ^ d; k = 0x6ed9eba1u; }
      else if (i < 60) { f = (bb & c) | (bb & d) | (c & d); k = 0x8f1bbcdcu; }
      else { f = bb ^ c ^ d; k = 0xca62c1d6u; }
      const uint32_t t = rotl(a, 5) + f + e + k + wi;
      e = d; d = c; c = rotl(bb, 30); bb = a; a = t;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e;
  }
  for (int i = 0; i < 20; ++i) put_hex(o + 2 * i, (h[i >> 2] >> (8 * (3 - (i & 3)))) & 0xff);
}

__device__ void sha256_row(const uint8_t* s, int32_t l, uint8_t* o, bool is224) {
  const int64_t total = ((int64_t)l + 8) / 64 * 64 + 64;
  uint32_t h[8];
  for (int i = 0; i < 8; ++i) h[i] = is224 ? kSha224H[i] : kSha256H[i];
  for (int64_t b = 0; b < total; b += 64) {
    uint32_t w[16];
    for (int j = 0; j < 16; ++j) {
      uint32_t v = 0;
      for (int q = 0; q < 4; ++q) v = (v << 8) | msg_byte<true>(s, l, b + 4 * j + q, total);
      w[j] = v;
    }
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      uint32_t wi;
      if (i < 16) wi = w[i];
      else {
        const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
        const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
        w[i & 15] = wi;
      }
      const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + kSha256K[i] + wi;
      const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      const uint32_t mj = (a & bb) ^ (a & c) ^ (bb & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
    }
    h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  const int nbytes = is224 ? 28 : 32;
  for (int i = 0; i < nbytes; ++i) put_hex(o + 2 * i, (h[i >> 2] >> (8 * (3 - (i & 3)))) & 0xff);
}

// kind: 0 md5, 1 sha1, 2 sha256, 3 sha224; row i → out[i * width …]
__global__ void __launch_bounds__(256) str_digest_kernel(const uint8_t* __restrict__ arena,
                                                         const int64_t* __restrict__ starts,
                                                         const int32_t* __restrict__ lens, int64_t n, int32_t kind,
                                                         int32_t width, uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* o = out + i * width;
    if (kind == 0) md5_row(s, l, o);
    else if (kind == 1) sha1_row(s, l, o);
    else sha256_row(s, l, o, kind == 3);
  }
}

__global__ void __launch_bounds__(256) str_crc32_kernel(const uint8_t* __restrict__ arena,
                                                        const int64_t* __restrict__ starts,
                                                        const int32_t* __restrict__ lens, int64_t n,
                                                        int64_t* __restrict__ out) {
  __shared__ uint32_t tab[256];
  for (int k = threadIdx.x; k < 256; k += blockDim.x) {
    uint32_t c = (uint32_t)k;
    for (int j = 0; j < 8; ++j) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    tab[k] = c;
  }
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint32_t c = 0xFFFFFFFFu;
    for (int32_t k = 0; k < l; ++k) c = tab[(c ^ s[k]) & 0xff] ^ (c >> 8);
    out[i] = (int64_t)(c ^ 0xFFFFFFFFu);
  }
}

// mode 0: upper-case hex of the bytes (2 per byte); mode 1: base64 with padding (4 per 3 bytes)
__global__ void __launch_bounds__(256) str_encode_kernel(const uint8_t* __restrict__ arena,
                                                         const int64_t* __restrict__ starts,
                                                         const int32_t* __restrict__ lens, int64_t n, int32_t mode,
                                                         const int64_t* __restrict__ out_starts,
                                                         uint8_t* __restrict__ out) {
  const char* hx = "0123456789ABCDEF";
  const char* b64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = arena + starts[i];
    const int32_t l = lens[i];
    uint8_t* o = out + out_starts[i];
    if (mode == 0) {
      for (int32_t k = 0; k < l; ++k) { o[2 * k] = hx[s[k] >> 4]; o[2 * k + 1] = hx[s[k] & 15]; }
    } else {
      int32_t k = 0, j = 0;
      for (; k + 3 <= l; k += 3, j += 4) {
        const uint32_t v = ((uint32_t)s[k] << 16) | ((uint32_t)s[k + 1] << 8) | s[k + 2];
        o[j] = b64[v >> 18]; o[j + 1] = b64[(v >> 12) & 63]; o[j + 2] = b64[(v >> 6) & 63]; o[j + 3] = b64[v & 63];
      }
      if (k < l) {
        const uint32_t v = ((uint32_t)s[k] << 16) | (k + 1 < l ? (uint32_t)s[k + 1] << 8 : 0u);
        o[j] = b64[v >> 18]; o[j + 1] = b64[(v >> 12) & 63];
        o[j + 2] = k + 1 < l ? b64[(v >> 6) & 63] : '=';
        o[j + 3] = '=';
      }
    }
  }
}

}  // namespace

DXA_API int dxa_str_digest(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n, int32_t kind,
                           uint8_t* out, void* st) {
  if (n <= 0) return 0;
  if (kind < 0 || kind > 3) return (int)hipErrorInvalidValue;
  const int32_t width = kind == 0 ? 32 : kind == 1 ? 40 : kind == 2 ? 64 : 56;
  hipLaunchKernelGGL(str_digest_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, kind, width, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_crc32(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n, int64_t* out,
                          void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_crc32_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, out);
  return (int)hipGetLastError();
}

DXA_API int dxa_str_encode(const uint8_t* arena, const int64_t* starts, const int32_t* lens, int64_t n, int32_t mode,
                           const int64_t* out_starts, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(str_encode_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, arena, starts, lens,
                     n, mode, out_starts, out);
  return (int)hipGetLastError();
}
