// Snappy codec (host): compressor for the producer side of the Kafka codec-2 path (simulated producers, tests) and
// the reference decoder for the host ingest path; format notes in dxa_snappy.h.
#include "dxa_snappy.h"

#include <cstring>
#include <vector>

namespace dxa {
namespace snappy {
namespace {

constexpr int64_t kFragment = 1 << 16;      // matches never reach across a 64 KiB fragment (2-byte offsets)
constexpr int64_t kXerialChunk = 32 * 1024;  // snappy-java's default block size
const uint8_t kMagic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};

inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

inline uint8_t* put_varint(uint8_t* d, uint64_t v) {
  while (v >= 128) {
    *d++ = (uint8_t)(v | 128);
    v >>= 7;
  }
  *d++ = (uint8_t)v;
  return d;
}

uint8_t* emit_literal(uint8_t* d, const uint8_t* s, int64_t len) {
  const int64_t n = len - 1;
  if (n < 60) {
    *d++ = (uint8_t)(n << 2);
  } else {
    int nb = n < (1 << 8) ? 1 : n < (1 << 16) ? 2 : n < (1 << 24) ? 3 : 4;
    *d++ = (uint8_t)((59 + nb) << 2);
    for (int k = 0; k < nb; ++k) *d++ = (uint8_t)(n >> (8 * k));
  }
  std::memcpy(d, s, (size_t)len);
  return d + len;
}

uint8_t* emit_copy(uint8_t* d, int64_t off, int64_t len) {
  while (len > 0) {
    // keep >= 4 bytes for a final copy-1 when splitting
    int64_t l = len > 64 ? (len - 64 < 4 ? 60 : 64) : len;
    if (l >= 4 && l <= 11 && off < 2048) {
      *d++ = (uint8_t)(1 | ((l - 4) << 2) | ((off >> 8) << 5));
      *d++ = (uint8_t)off;
    } else {
      *d++ = (uint8_t)(2 | ((l - 1) << 2));
      *d++ = (uint8_t)off;
      *d++ = (uint8_t)(off >> 8);
    }
    len -= l;
  }
  return d;
}

uint8_t* compress_fragment(const uint8_t* s, int64_t n, uint8_t* d, std::vector<uint16_t>& table) {
  const int hbits = 14;
  std::fill(table.begin(), table.end(), 0);
  int64_t lit = 0, i = 0;
  if (n >= 15) {
    const int64_t limit = n - 4;
    i = 1;
    while (i < limit) {
      const uint32_t v = load32(s + i);
      const uint32_t h = (v * 0x1e35a7bdu) >> (32 - hbits);
      const int64_t cand = table[h];
      table[h] = (uint16_t)i;
      if (cand < i && load32(s + cand) == v) {
        int64_t len = 4;
        while (i + len < n && s[cand + len] == s[i + len]) ++len;
        if (i > lit) d = emit_literal(d, s + lit, i - lit);
        d = emit_copy(d, i - cand, len);
        i += len;
        lit = i;
        if (i < limit) table[(load32(s + i - 1) * 0x1e35a7bdu) >> (32 - hbits)] = (uint16_t)(i - 1);
      } else {
        ++i;
      }
    }
  }
  if (n > lit) d = emit_literal(d, s + lit, n - lit);
  return d;
}

inline int32_t be32(const uint8_t* p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}
inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

}  // namespace

int64_t max_compressed_length(int64_t n) { return 32 + n + n / 6; }

int64_t compress_raw(const uint8_t* src, int64_t n, uint8_t* dst) {
  uint8_t* d = put_varint(dst, (uint64_t)n);
  std::vector<uint16_t> table(1 << 14);
  for (int64_t f = 0; f < n; f += kFragment) {
    const int64_t m = n - f < kFragment ? n - f : kFragment;
    d = compress_fragment(src + f, m, d, table);
  }
  return d - dst;
}

int64_t raw_length(const uint8_t* src, int64_t n, int32_t* hdr) {
  uint64_t v = 0;
  int shift = 0;
  for (int64_t k = 0; k < n && k < 5; ++k) {
    v |= (uint64_t)(src[k] & 127) << shift;
    if (!(src[k] & 128)) {
      if (hdr) *hdr = (int32_t)(k + 1);
      // the declared length is untrusted: no element expands more than a 3-byte copy of 64 bytes does, so a block of
      // c element bytes decodes to at most c*64/3 (+ one copy's slack); a larger claim is corrupt and must not size
      // an allocation
      const uint64_t body = (uint64_t)(n - (k + 1));
      if (v > body * 64 / 3 + 64) return -1;
      return v > 0x7fffffffull ? -1 : (int64_t)v;
    }
    shift += 7;
  }
  return -1;
}

int64_t decompress_raw(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int32_t hdr = 0;
  const int64_t total = raw_length(src, n, &hdr);
  if (total < 0 || total > cap) return -1;
  int64_t ip = hdr, op = 0;
  while (ip < n) {
    const uint32_t tag = src[ip++];
    const uint32_t kind = tag & 3;
    if (kind == 0) {
      int64_t len = (tag >> 2) + 1;
      if ((tag >> 2) >= 60) {
        const int nb = (int)(tag >> 2) - 59;
        if (ip + nb > n) return -1;
        len = 0;
        for (int k = 0; k < nb; ++k) len |= (int64_t)src[ip + k] << (8 * k);
        len += 1;
        ip += nb;
      }
      if (len > n - ip || len > total - op) return -1;
      std::memcpy(dst + op, src + ip, (size_t)len);
      ip += len;
      op += len;
      continue;
    }
    int64_t len, off;
    if (kind == 1) {
      if (ip >= n) return -1;
      len = ((tag >> 2) & 7) + 4;
      off = ((int64_t)(tag >> 5) << 8) | src[ip++];
    } else if (kind == 2) {
      if (ip + 2 > n) return -1;
      len = (tag >> 2) + 1;
      off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) return -1;
      len = (tag >> 2) + 1;
      off = (int64_t)load32(src + ip);
      ip += 4;
    }
    if (off == 0 || off > op || len > total - op) return -1;
    for (int64_t k = 0; k < len; ++k) dst[op + k] = dst[op - off + k];
    op += len;
  }
  return op == total ? op : -1;
}

bool is_xerial(const uint8_t* src, int64_t n) { return n >= 16 && std::memcmp(src, kMagic, 8) == 0; }

int64_t xerial_bound(int64_t n) {
  return 16 + (n + kXerialChunk - 1) / kXerialChunk * (4 + 32) + n + n / 6 + 32;
}

int64_t xerial_compress(const uint8_t* src, int64_t n, uint8_t* dst) {
  std::memcpy(dst, kMagic, 8);
  put_be32(dst + 8, 1);
  put_be32(dst + 12, 1);
  int64_t o = 16;
  for (int64_t f = 0; f < n; f += kXerialChunk) {
    const int64_t m = n - f < kXerialChunk ? n - f : kXerialChunk;
    const int64_t c = compress_raw(src + f, m, dst + o + 4);
    put_be32(dst + o, (uint32_t)c);
    o += 4 + c;
  }
  return o;
}

int64_t xerial_chunks(const uint8_t* src, int64_t n, int64_t* off, int32_t* len, int64_t* out_len, int64_t max) {
  if (!is_xerial(src, n)) return -1;
  int64_t p = 16, k = 0;
  while (p < n) {
    if (n - p < 4) return -1;
    const int32_t c = be32(src + p);
    if (c < 0 || c > n - p - 4) return -1;
    const int64_t u = raw_length(src + p + 4, c, nullptr);
    if (u < 0) return -1;
    if (off && k < max) {
      off[k] = p + 4;
      len[k] = c;
      out_len[k] = u;
    }
    ++k;
    p += 4 + c;
  }
  return k;
}

int64_t payload_length(const uint8_t* src, int64_t n) {
  if (!is_xerial(src, n)) return raw_length(src, n, nullptr);
  const int64_t nc = xerial_chunks(src, n, nullptr, nullptr, nullptr, 0);
  if (nc < 0) return -1;
  std::vector<int64_t> off((size_t)nc), out((size_t)nc);
  std::vector<int32_t> len((size_t)nc);
  xerial_chunks(src, n, off.data(), len.data(), out.data(), nc);
  int64_t t = 0;
  for (int64_t v : out) t += v;
  return t;
}

int64_t decompress_payload(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  if (!is_xerial(src, n)) return decompress_raw(src, n, dst, cap);
  const int64_t nc = xerial_chunks(src, n, nullptr, nullptr, nullptr, 0);
  if (nc < 0) return -1;
  std::vector<int64_t> off((size_t)nc), out((size_t)nc);
  std::vector<int32_t> len((size_t)nc);
  xerial_chunks(src, n, off.data(), len.data(), out.data(), nc);
  int64_t o = 0;
  for (int64_t k = 0; k < nc; ++k) {
    const int64_t m = decompress_raw(src + off[k], len[k], dst + o, cap - o);
    if (m < 0) return -1;
    o += m;
  }
  return o;
}

}  // namespace snappy
}  // namespace dxa

extern "C" {

__attribute__((visibility("default"))) int64_t dxa_snappy_compress(const uint8_t* src, int64_t n, uint8_t* dst,
                                                                   int64_t cap, int32_t xerial) {
  const int64_t need = xerial ? dxa::snappy::xerial_bound(n) : dxa::snappy::max_compressed_length(n);
  if (cap < need) return -need;
  return xerial ? dxa::snappy::xerial_compress(src, n, dst) : dxa::snappy::compress_raw(src, n, dst);
}

__attribute__((visibility("default"))) int64_t dxa_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst,
                                                                     int64_t cap) {
  return dxa::snappy::decompress_payload(src, n, dst, cap);
}

__attribute__((visibility("default"))) int64_t dxa_snappy_length(const uint8_t* src, int64_t n) {
  return dxa::snappy::payload_length(src, n);
}

}  // extern "C"
