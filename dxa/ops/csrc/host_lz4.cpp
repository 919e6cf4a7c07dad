// Host LZ4 codec (see dxa_lz4.h): greedy hash-chain-free compressor with backward match extension, bounds-checked
// decompressor, and the frame container.  Used by the Kafka codec (compression type 3), the simulated-data
// producer and the compressed-ingest path whose blocks the GPU decodes (lz4.hip).
#include "dxa_lz4.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace dxa {
namespace lz4 {
namespace {

constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMfLimit = 12;
constexpr int kHashLog = 16;
constexpr uint32_t kFrameMagic = 0x184D2204u;

inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }
inline void wr32le(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }
inline uint32_t rd32le(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

inline uint8_t* put_len(uint8_t* op, int64_t len) {
  while (len >= 255) { *op++ = 255; len -= 255; }
  *op++ = (uint8_t)len;
  return op;
}

inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// Decode with matches allowed to reach back to base (dependent-block frames decode into one contiguous output).
int64_t decode(const uint8_t* src, int64_t n, uint8_t* base, int64_t pos, int64_t cap) {
  const uint8_t* ip = src;
  const uint8_t* iend = src + n;
  int64_t op = pos;
  while (ip < iend) {
    const uint8_t token = *ip++;
    int64_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do { if (ip >= iend) return -1; b = *ip++; lit += b; } while (b == 255);
    }
    if (lit > iend - ip || lit > cap - op) return -1;
    std::memcpy(base + op, ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (ip >= iend) break;                       // last sequence: literals only
    if (iend - ip < 2) return -1;
    const int64_t off = (int64_t)ip[0] | (int64_t)ip[1] << 8;
    ip += 2;
    if (off == 0 || off > op) return -1;
    int64_t ml = (token & 15);
    if (ml == 15) {
      uint8_t b;
      do { if (ip >= iend) return -1; b = *ip++; ml += b; } while (b == 255);
    }
    ml += kMinMatch;
    if (ml > cap - op) return -1;
    uint8_t* d = base + op;
    const uint8_t* s = d - off;
    if (off >= ml) std::memcpy(d, s, (size_t)ml);
    else for (int64_t k = 0; k < ml; ++k) d[k] = s[k];   // overlapping copy repeats the pattern
    op += ml;
  }
  return op - pos;
}

int bd_id(int32_t block_size) {
  if (block_size <= 64 * 1024) return 4;
  if (block_size <= 256 * 1024) return 5;
  if (block_size <= 1024 * 1024) return 6;
  return 7;
}

}  // namespace

int64_t block_bound(int64_t n) { return n + n / 255 + 16; }

int64_t compress_block(const uint8_t* src, int64_t n, uint8_t* dst) {
  uint8_t* op = dst;
  int64_t anchor = 0;
  if (n >= kMfLimit + 1) {
    std::vector<int32_t> table(1u << kHashLog, -1);
    const int64_t match_limit = n - kLastLiterals;
    const int64_t search_limit = n - kMfLimit;
    int64_t ip = 0;
    int64_t misses = 0;
    while (ip < search_limit) {
      const uint32_t seq = rd32(src + ip);
      const uint32_t h = hash4(seq);
      const int64_t ref = table[h];
      table[h] = (int32_t)ip;
      if (ref < 0 || ip - ref > 65535 || rd32(src + ref) != seq) {
        ip += 1 + (misses++ >> 6);               // skip faster through incompressible stretches
        continue;
      }
      misses = 0;
      int64_t s = ip, r = ref;
      while (s > anchor && r > 0 && src[s - 1] == src[r - 1]) { --s; --r; }
      int64_t len = kMinMatch + (ip - s);
      while (s + len < match_limit && src[r + len] == src[s + len]) ++len;
      const int64_t lit = s - anchor;
      uint8_t* token = op++;
      const int64_t mlc = len - kMinMatch;
      *token = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mlc >= 15 ? 15 : mlc));
      if (lit >= 15) op = put_len(op, lit - 15);
      std::memcpy(op, src + anchor, (size_t)lit);
      op += lit;
      const int64_t off = s - r;
      *op++ = (uint8_t)off;
      *op++ = (uint8_t)(off >> 8);
      if (mlc >= 15) op = put_len(op, mlc - 15);
      ip = s + len;
      anchor = ip;
      if (ip - 2 >= 0 && ip - 2 < search_limit) table[hash4(rd32(src + ip - 2))] = (int32_t)(ip - 2);
    }
  }
  const int64_t lit = n - anchor;
  *op++ = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
  if (lit >= 15) op = put_len(op, lit - 15);
  if (lit) std::memcpy(op, src + anchor, (size_t)lit);
  op += lit;
  return op - dst;
}

// High-compression block: hash chains over the block (every position inserted), longest match among up to `depth`
// candidates, one-step lazy evaluation.  Same output format as compress_block.
int64_t compress_block_hc(const uint8_t* src, int64_t n, uint8_t* dst, int depth) {
  uint8_t* op = dst;
  int64_t anchor = 0;
  if (n >= kMfLimit + 1) {
    std::vector<int32_t> head(1u << kHashLog, -1);
    std::vector<int32_t> chain((size_t)n, -1);
    const int64_t match_limit = n - kLastLiterals;
    const int64_t search_limit = n - kMfLimit;
    int64_t next_insert = 0;
    auto insert_upto = [&](int64_t pos) {
      for (; next_insert < pos; ++next_insert) {
        const uint32_t h = hash4(rd32(src + next_insert));
        chain[next_insert] = head[h];
        head[h] = (int32_t)next_insert;
      }
    };
    auto find = [&](int64_t ip, int64_t& best_ref) -> int64_t {
      insert_upto(ip);
      const uint32_t seq = rd32(src + ip);
      int64_t best = 0;
      int64_t cand = head[hash4(seq)];
      for (int d = 0; d < depth && cand >= 0 && ip - cand <= 65535; ++d, cand = chain[cand]) {
        if (rd32(src + cand) != seq) continue;
        int64_t len = kMinMatch;
        while (ip + len < match_limit && src[cand + len] == src[ip + len]) ++len;
        if (len > best) {
          best = len;
          best_ref = cand;
          if (ip + len >= match_limit) break;
        }
      }
      return best;
    };
    int64_t ip = 0;
    while (ip < search_limit) {
      int64_t ref = -1;
      int64_t len = find(ip, ref);
      if (len < kMinMatch) { ++ip; continue; }
      while (ip + 1 < search_limit) {                  // lazy: a longer match one byte later wins
        int64_t ref2 = -1;
        const int64_t len2 = find(ip + 1, ref2);
        if (len2 <= len) break;
        ++ip;
        len = len2;
        ref = ref2;
      }
      int64_t s = ip, r = ref;
      while (s > anchor && r > 0 && src[s - 1] == src[r - 1]) { --s; --r; ++len; }
      const int64_t lit = s - anchor;
      uint8_t* token = op++;
      const int64_t mlc = len - kMinMatch;
      *token = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (mlc >= 15 ? 15 : mlc));
      if (lit >= 15) op = put_len(op, lit - 15);
      std::memcpy(op, src + anchor, (size_t)lit);
      op += lit;
      const int64_t off = s - r;
      *op++ = (uint8_t)off;
      *op++ = (uint8_t)(off >> 8);
      if (mlc >= 15) op = put_len(op, mlc - 15);
      ip = s + len;
      anchor = ip;
    }
  }
  const int64_t lit = n - anchor;
  *op++ = (uint8_t)((lit >= 15 ? 15 : lit) << 4);
  if (lit >= 15) op = put_len(op, lit - 15);
  if (lit) std::memcpy(op, src + anchor, (size_t)lit);
  op += lit;
  return op - dst;
}

int64_t decompress_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) { return decode(src, n, dst, 0, cap); }

uint32_t xxh32(const uint8_t* p, int64_t n, uint32_t seed) {
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
  const uint8_t* end = p + n;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 16;
    do {
      v1 = rotl(v1 + rd32le(p) * P2, 13) * P1; p += 4;
      v2 = rotl(v2 + rd32le(p) * P2, 13) * P1; p += 4;
      v3 = rotl(v3 + rd32le(p) * P2, 13) * P1; p += 4;
      v4 = rotl(v4 + rd32le(p) * P2, 13) * P1; p += 4;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)n;
  while (end - p >= 4) { h = rotl(h + rd32le(p) * P3, 17) * P4; p += 4; }
  while (p < end) { h = rotl(h + (*p++) * P5, 11) * P1; }
  h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
  return h;
}

int64_t frame_bound(int64_t n, int32_t block_size) {
  const int64_t nb = (n + block_size - 1) / block_size;
  return 19 + nb * (4 + block_bound(block_size)) + 4;
}

int64_t compress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t block_size, int32_t threads,
                       int32_t level) {
  if (block_size <= 0 || block_size > 4 * 1024 * 1024) return -1;
  if (cap < frame_bound(n, block_size)) return -1;
  uint8_t* op = dst;
  wr32le(op, kFrameMagic); op += 4;
  uint8_t* desc = op;
  *op++ = 0x40 | 0x20 | 0x08;                    // version 01, independent blocks, content size present
  *op++ = (uint8_t)(bd_id(block_size) << 4);
  for (int k = 0; k < 8; ++k) *op++ = (uint8_t)((uint64_t)n >> (8 * k));
  *op = (uint8_t)((xxh32(desc, op - desc, 0) >> 8) & 0xff);
  ++op;
  const int64_t nb = (n + block_size - 1) / block_size;
  std::vector<int64_t> clen(nb);
  std::vector<uint8_t> tmp((size_t)(nb * block_bound(block_size)));
  auto work = [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const int64_t s = b * block_size;
      const int64_t len = std::min<int64_t>(block_size, n - s);
      uint8_t* out = tmp.data() + b * block_bound(block_size);
      clen[b] = level <= 2 ? compress_block(src + s, len, out)
                           : compress_block_hc(src + s, len, out, 1 << std::min(level - 1, 12));
    }
  };
  const int T = std::max(1, std::min<int>(threads, (int)std::min<int64_t>(nb, 64)));
  if (T == 1) {
    work(0, nb);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t) ts.emplace_back(work, nb * t / T, nb * (t + 1) / T);
    for (auto& t : ts) t.join();
  }
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t s = b * block_size;
    const int64_t len = std::min<int64_t>(block_size, n - s);
    if (clen[b] >= len) {                         // incompressible: store
      wr32le(op, (uint32_t)len | 0x80000000u); op += 4;
      std::memcpy(op, src + s, (size_t)len); op += len;
    } else {
      wr32le(op, (uint32_t)clen[b]); op += 4;
      std::memcpy(op, tmp.data() + b * block_bound(block_size), (size_t)clen[b]); op += clen[b];
    }
  }
  wr32le(op, 0); op += 4;
  return op - dst;
}

int64_t frame_blocks(const uint8_t* src, int64_t n, int64_t* comp_off, int32_t* comp_len, uint8_t* stored,
                     int64_t max_blocks, int64_t* content_size, int32_t* max_block_size, int64_t* frame_end) {
  if (n < 7 || rd32le(src) != kFrameMagic) return -1;
  const uint8_t flg = src[4], bd = src[5];
  if ((flg >> 6) != 1) return -1;
  const bool indep = (flg >> 5) & 1, bsum = (flg >> 4) & 1, csize = (flg >> 3) & 1, csum = (flg >> 2) & 1,
             dict = flg & 1;
  if (dict) return -2;
  int64_t p = 6;
  *content_size = -1;
  if (csize) {
    if (n < p + 8) return -1;
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v |= (uint64_t)src[p + k] << (8 * k);
    *content_size = (int64_t)v;
    p += 8;
  }
  p += 1;                                         // header checksum (not enforced: old Kafka clients wrote it wrong)
  const int id = (bd >> 4) & 7;
  *max_block_size = id >= 4 ? (1 << (2 * id + 8)) : 4 * 1024 * 1024;
  int64_t nb = 0;
  while (true) {
    if (n < p + 4) return -1;
    const uint32_t w = rd32le(src + p);
    p += 4;
    if (w == 0) break;
    const int64_t len = w & 0x7fffffffu;
    if (n < p + len) return -1;
    if (nb < max_blocks && comp_off) {
      comp_off[nb] = p;
      comp_len[nb] = (int32_t)len;
      stored[nb] = (uint8_t)(w >> 31);
    }
    ++nb;
    p += len + (bsum ? 4 : 0);
  }
  if (csum) p += 4;
  if (frame_end) *frame_end = p;
  return indep ? nb : -2;
}

int64_t decompress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int64_t out = 0, p = 0;
  while (p < n) {
    const uint8_t* f = src + p;
    const int64_t m = n - p;
    if (m < 7 || rd32le(f) != kFrameMagic) return -1;
    const uint8_t flg = f[4];
    if (flg & 1) return -2;
    const bool bsum = (flg >> 4) & 1, csize = (flg >> 3) & 1, csum = (flg >> 2) & 1;
    int64_t q = 6 + (csize ? 8 : 0) + 1;
    while (true) {
      if (m < q + 4) return -1;
      const uint32_t w = rd32le(f + q);
      q += 4;
      if (w == 0) break;
      const int64_t len = w & 0x7fffffffu;
      if (m < q + len) return -1;
      if (w >> 31) {
        if (len > cap - out) return -1;
        std::memcpy(dst + out, f + q, (size_t)len);
        out += len;
      } else {
        const int64_t r = decode(f + q, len, dst, out, cap);   // dependent blocks may reach into earlier output
        if (r < 0) return -1;
        out += r;
      }
      q += len + (bsum ? 4 : 0);
    }
    if (csum) q += 4;
    p += q;
  }
  return out;
}

}  // namespace lz4
}  // namespace dxa

extern "C" {
#define DXA_API __attribute__((visibility("default")))
DXA_API int64_t dxa_lz4_frame_bound(int64_t n, int32_t block_size) { return dxa::lz4::frame_bound(n, block_size); }
DXA_API int64_t dxa_lz4_compress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t block_size,
                                       int32_t threads) {
  return dxa::lz4::compress_frame(src, n, dst, cap, block_size, threads, 0);
}
DXA_API int64_t dxa_lz4_compress_frame_level(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap,
                                             int32_t block_size, int32_t threads, int32_t level) {
  return dxa::lz4::compress_frame(src, n, dst, cap, block_size, threads, level);
}
DXA_API int64_t dxa_lz4_decompress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  return dxa::lz4::decompress_frame(src, n, dst, cap);
}
DXA_API int64_t dxa_lz4_frame_blocks(const uint8_t* src, int64_t n, int64_t* comp_off, int32_t* comp_len,
                                     uint8_t* stored, int64_t max_blocks, int64_t* content_size,
                                     int32_t* max_block_size, int64_t* frame_end) {
  return dxa::lz4::frame_blocks(src, n, comp_off, comp_len, stored, max_blocks, content_size, max_block_size,
                                frame_end);
}
DXA_API int64_t dxa_lz4_compress_block(const uint8_t* src, int64_t n, uint8_t* dst) {
  return dxa::lz4::compress_block(src, n, dst);
}
DXA_API int64_t dxa_lz4_decompress_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  return dxa::lz4::decompress_block(src, n, dst, cap);
}
DXA_API uint32_t dxa_xxh32(const uint8_t* p, int64_t n, uint32_t seed) { return dxa::lz4::xxh32(p, n, seed); }
}
