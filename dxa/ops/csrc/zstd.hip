// Zstandard (RFC 8878) frame decoder for gfx950: zstd-compressed Kafka record batches (codec 4 — the records section
// of a batch is one frame, as zstd-jni's ZstdOutputStream writes it: no content size, so the planner gives every
// frame a capacity slot of blocks x block maximum and this kernel reports the decoded size) are decompressed in HBM
// after a compressed H2D copy.  At ~4.5x on SimulatedData batches zstd moves ~40 % fewer PCIe bytes per event than
// LZ4 (2.7x), which is what bounds the Kafka ingest.
//
// Layout: ZG = 32 lanes own one frame (2 frames per 64-thread workgroup).  A frame's blocks share the window,
// the repeat offsets and the entropy tables (treeless literals, repeat-mode sequence tables), so one group decodes
// the whole frame in order.  The entropy decoding is a serial chain per bitstream, so the group runs it redundantly
// on group-uniform state; the lanes split what is parallel:
//   * Huffman literals: the four streams of a 4-stream literals section are decoded by lanes 0..3 at once (one
//     stream each, same instruction stream), into the TAIL of the frame's output slot — sequence execution then
//     moves them forward (the output position never passes the unread literal, so no scratch buffer is needed);
//   * Huffman decode-table fill (2^maxBits entries), raw / RLE block copies, literal runs and match copies, ZG bytes
//     per step.  A match copy reads dst[s + (i mod off)], which is always before the copy's own start, so a copy has
//     no internal dependency; a `s_waitcnt vmcnt(0)` makes the group's earlier stores visible only when a source
//     reaches past the output known complete at the last wait (as lz4.hip / inflate.hip).
//   * Tables live in LDS per group: the Huffman table (2048 x u16), the LL / ML / OF FSE tables (512 / 512 / 256
//     cells of base | symbol | bits) and the Huffman-weight FSE table — 9.7 KiB per frame, 16 frames per CU (the
//     180-VGPR kernel runs 2 waves per SIMD).
// Bit reading: a 64-bit container over the backward bitstream (zstd's BIT_DStream shape): n bits are the container's
// top bits after `consumed`, reloaded from 8 bytes further back when more than 64 would be needed; bits below the
// stream start read as zeros and leave the remaining count negative (the overflow the weight decoder and the
// end-of-stream checks test).
// Every size, offset, table index and input position is checked; a malformed frame stops with a nonzero status
// (the Kafka source then rejects the batch), never an out-of-range access.  The content checksum is not verified
// (the batch's CRC-32C covers the bytes in transit).
#include "dxa_common.h"

namespace {

// lanes per frame: 32, two frames per wave (profiles/round6/codecs/README.md: 16 lanes put 4 divergent frames in a
// wave at one wave per SIMD; 32 halves the divergence and doubles the waves per SIMD for the same frames per CU)
#ifndef DXA_ZSTD_ZG
#define DXA_ZSTD_ZG 32
#endif
constexpr int ZG = DXA_ZSTD_ZG;         // a power of two, at most a wave
constexpr uint64_t kGroupMask = ZG == 64 ? ~0ull : ((1ull << ZG) - 1);
constexpr int ZWG = 64;                 // threads per workgroup: ZWG / ZG frames
constexpr int kWaitVm0 = 0xF70;         // s_waitcnt vmcnt(0) (gfx9 encoding)
constexpr int32_t kBlockMax = 128 * 1024;

enum : int32_t {
  Z_OK = 0, Z_TRUNC = 1, Z_OFFSET = 2, Z_OVERFLOW = 3, Z_SIZE = 4, Z_HEADER = 5, Z_HUF = 6, Z_FSE = 7, Z_SEQ = 8,
  Z_LIT = 9, Z_BLOCK = 10
};

struct ZTables {
  uint16_t huf[2048];                   // (bits << 8) | symbol
  uint32_t ll[512];                     // (base << 16) | (symbol << 8) | bits
  uint32_t ml[512];
  uint32_t of[256];
  uint32_t wt[64];                      // Huffman-weight FSE table (accuracy <= 6)
  int16_t norm[64];                     // normalized counts being built
  uint16_t nxt[64];
  uint8_t w[256];                       // Huffman weights
};

__constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2,
                                   2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   -1, -1, -1, -1, -1};
__constant__ uint32_t kLLBase[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28,
                                     32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                                    4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24,
                                     25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void stores_visible() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int highbit32(uint32_t v) { return 31 - __builtin_clz(v); }

typedef uint64_t u64u __attribute__((aligned(1)));

// Bytes [p, p + 8) little-endian; the caller guarantees they lie inside the frame (or its 32-byte tail pad).
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }

// Backward bitstream over [start, start + n).
struct BitB {
  const uint8_t* start;
  const uint8_t* ptr;
  uint64_t c;
  int32_t used;                         // bits consumed from the top of c
  int32_t pad;                          // zero bits below the stream start at the bottom of c (streams < 8 bytes)
  __device__ bool init(const uint8_t* s, int32_t n) {
    start = s;
    if (n <= 0) return false;
    const uint32_t last = s[n - 1];
    if (last == 0) return false;
    used = 8 - highbit32(last);         // the zero bits above the end marker, and the marker
    if (n >= 8) {
      ptr = s + n - 8;
      c = ld64(ptr);
      pad = 0;
    } else {
      ptr = s;
      uint64_t v = 0;
      for (int k = 0; k < n; ++k) v |= (uint64_t)s[k] << (8 * k);
      c = v << (8 * (8 - n));            // the stream's bytes at the top, as an 8-byte load would hold them
      pad = 8 * (8 - n);
    }
    return true;
  }
  // bits remaining (negative once more were read than the stream holds)
  __device__ __forceinline__ int32_t left() const { return (int32_t)(ptr - start) * 8 + 64 - used - pad; }
  __device__ __forceinline__ void reload() {
    if (used < 8) return;
    int32_t nb = used >> 3;
    const int32_t room = (int32_t)(ptr - start);
    if (nb > room) nb = room;
    if (nb == 0) return;
    ptr -= nb;
    used -= 8 * nb;
    c = ld64(ptr);
  }
  __device__ __forceinline__ uint32_t peek(int k) const {
    if (k == 0 || used >= 64) return 0;
    return (uint32_t)((c << used) >> (64 - k));
  }
  __device__ __forceinline__ uint32_t read(int k) {
    if (k == 0) return 0;
    if (used + k > 64) reload();
    const uint32_t v = peek(k);
    used += k;
    return v;
  }
};

// Forward bit reader for FSE table descriptions (little-endian from the start), bounded by n bytes.
struct BitF {
  const uint8_t* p;
  int32_t n;
  int32_t bit;
  __device__ uint32_t peek(int k) const {
    uint32_t v = 0;
    const int32_t b0 = bit >> 3;
    uint64_t w = 0;
    for (int j = 0; j < 5; ++j) {
      const int32_t q = b0 + j;
      if (q < n) w |= (uint64_t)p[q] << (8 * j);
    }
    v = (uint32_t)(w >> (bit & 7));
    return k >= 32 ? v : (v & ((1u << k) - 1u));
  }
  __device__ void skip(int k) { bit += k; }
  __device__ uint32_t read(int k) {
    const uint32_t v = peek(k);
    bit += k;
    return v;
  }
};

// FSE table description → T.norm; returns bytes consumed, or -1.
__device__ int32_t read_counts(const uint8_t* src, int32_t n, int max_log, int max_sym, ZTables& T, int* nsym,
                               int* log) {
  BitF r{src, n, 0};
  const int al = (int)r.read(4) + 5;
  if (al > max_log) return -1;
  int remaining = (1 << al) + 1;
  int threshold = 1 << al;
  int nbits = al + 1;
  int s = 0;
  bool prev0 = false;
  while (remaining > 1 && s <= max_sym) {
    if (prev0) {
      int n0 = s;
      while (r.peek(16) == 0xFFFFu) {
        n0 += 24;
        r.skip(16);
        if (n0 > max_sym + 1) return -1;
      }
      while ((r.peek(2) & 3u) == 3u) { n0 += 3; r.skip(2); }
      n0 += (int)r.read(2);
      if (n0 > max_sym + 1) return -1;
      while (s < n0) T.norm[s++] = 0;
      if (s > max_sym) break;
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    const uint32_t low = r.peek(nbits - 1) & (uint32_t)(threshold - 1);
    if ((int)low < max) {
      count = (int)low;
      r.skip(nbits - 1);
    } else {
      count = (int)(r.peek(nbits) & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      r.skip(nbits);
    }
    count -= 1;
    remaining -= count < 0 ? -count : count;
    T.norm[s++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
    if (r.bit > 8 * n) return -1;
  }
  if (remaining != 1 || s > max_sym + 1) return -1;
  *nsym = s;
  *log = al;
  const int32_t used = (r.bit + 7) >> 3;
  return used <= n ? used : -1;
}

// Decode table from T.norm into `tab` (cells of (base << 16) | (sym << 8) | bits).  Every lane of the group runs
// it (same values, so each lane reads back what it wrote); false for an inconsistent distribution.
__device__ bool build_fse(ZTables& T, int nsym, int log, uint32_t* tab) {
  const int size = 1 << log;
  int high = size - 1;
  for (int s = 0; s < nsym; ++s) {
    if (T.norm[s] == -1) {
      if (high < 0) return false;
      tab[high--] = (uint32_t)s << 8;
      T.nxt[s] = 1;
    } else {
      T.nxt[s] = (uint16_t)T.norm[s];
    }
  }
  const int step = (size >> 1) + (size >> 3) + 3;
  int pos = 0;
  if (high < 0) return false;
  int placed = 0;
  for (int s = 0; s < nsym; ++s) {
    const int cnt = T.norm[s];
    placed += cnt > 0 ? cnt : 0;
    if (placed > high + 1) return false;                  // more cells than the table holds
    for (int i = 0; i < cnt; ++i) {
      tab[pos] = (uint32_t)s << 8;
      do { pos = (pos + step) & (size - 1); } while (pos > high);
    }
  }
  if (pos != 0) return false;
  for (int c = 0; c < size; ++c) {
    const int s = (int)((tab[c] >> 8) & 0xff);
    const uint32_t x = T.nxt[s];
    T.nxt[s] = (uint16_t)(x + 1);
    if (x == 0) return false;
    const int nb = log - highbit32(x);
    tab[c] = (((x << nb) - (uint32_t)size) << 16) | ((uint32_t)s << 8) | (uint32_t)nb;
  }
  return true;
}

__device__ bool build_default(ZTables& T, const int16_t* def, int nsym, int log, uint32_t* tab) {
  for (int s = 0; s < nsym; ++s) T.norm[s] = def[s];
  return build_fse(T, nsym, log, tab);
}

// Sequence table for one symbol kind by its mode; returns bytes consumed or -1.  *log / *valid track the table.
__device__ int32_t seq_table(int mode, const uint8_t* src, int32_t n, const int16_t* def, int def_n, int def_log,
                             int max_log, int max_sym, ZTables& T, uint32_t* tab, int* log, bool* valid) {
  if (mode == 0) {
    if (!build_default(T, def, def_n, def_log, tab)) return -1;
    *log = def_log;
    *valid = true;
    return 0;
  }
  if (mode == 1) {
    if (n < 1 || src[0] > max_sym) return -1;
    tab[0] = (uint32_t)src[0] << 8;
    *log = 0;
    *valid = true;
    return 1;
  }
  if (mode == 2) {
    int nsym = 0, lg = 0;
    const int32_t d = read_counts(src, n, max_log, max_sym, T, &nsym, &lg);
    if (d < 0 || !build_fse(T, nsym, lg, tab)) return -1;
    *log = lg;
    *valid = true;
    return d;
  }
  return *valid ? 0 : -1;
}

// Huffman tree description → T.huf (lanes split the fill); returns bytes consumed, or -1.  *max_bits out.
__device__ int32_t read_huffman(const uint8_t* src, int32_t n, ZTables& T, int gl, int* max_bits) {
  if (n < 1) return -1;
  const int hb = src[0];
  int nw = 0;
  int32_t used;
  if (hb < 128) {
    if (hb + 1 > n) return -1;
    int nsym = 0, lg = 0;
    const int32_t d = read_counts(src + 1, hb, 6, 63, T, &nsym, &lg);
    if (d < 0 || !build_fse(T, nsym, lg, T.wt)) return -1;
    BitB b;
    if (!b.init(src + 1 + d, hb - d)) return -1;
    uint32_t s1 = b.read(lg), s2 = b.read(lg);
    while (true) {
      if (nw + 2 > 255) return -1;
      uint32_t e = T.wt[s1];
      T.w[nw++] = (uint8_t)(e >> 8);
      s1 = (e >> 16) + b.read((int)(e & 0xff));
      if (b.left() < 0) { T.w[nw++] = (uint8_t)(T.wt[s2] >> 8); break; }
      e = T.wt[s2];
      T.w[nw++] = (uint8_t)(e >> 8);
      s2 = (e >> 16) + b.read((int)(e & 0xff));
      if (b.left() < 0) { T.w[nw++] = (uint8_t)(T.wt[s1] >> 8); break; }
    }
    used = 1 + hb;
  } else {
    nw = hb - 127;
    const int32_t bytes = (nw + 1) / 2;
    if (1 + bytes > n) return -1;
    for (int i = 0; i < nw; ++i) {
      const uint32_t x = src[1 + i / 2];
      T.w[i] = (uint8_t)((i & 1) ? (x & 15) : (x >> 4));
    }
    used = 1 + bytes;
  }
  uint32_t sum = 0;
  uint32_t cnt[13];
  for (int k = 0; k < 13; ++k) cnt[k] = 0;
  for (int i = 0; i < nw; ++i) {
    const int wv = T.w[i];
    if (wv > 11) return -1;
    if (wv) sum += 1u << (wv - 1);
    ++cnt[wv];
  }
  if (sum == 0) return -1;
  const int maxb = highbit32(sum) + 1;
  if (maxb > 11) return -1;
  const uint32_t rest = (1u << maxb) - sum;
  if (rest & (rest - 1)) return -1;
  const int lastw = highbit32(rest) + 1;
  T.w[nw++] = (uint8_t)lastw;
  ++cnt[lastw];
  uint32_t start[13];
  uint32_t pos = 0;
  for (int k = 1; k <= maxb; ++k) {
    start[k] = pos;
    pos += cnt[k] << (k - 1);
  }
  if (pos != (1u << maxb)) return -1;
  // fill: symbol by symbol (weights ascending, then symbol order), each symbol's run split over the lanes
  for (int i = 0; i < nw; ++i) {
    const int k = T.w[i];
    if (!k) continue;
    const uint32_t len = 1u << (k - 1);
    const uint16_t e = (uint16_t)(((maxb + 1 - k) << 8) | i);
    for (uint32_t j = (uint32_t)gl; j < len; j += ZG) T.huf[start[k] + j] = e;
    start[k] += len;
  }
  lane_sync();
  *max_bits = maxb;
  return used;
}

// One Huffman stream of `count` literals into out[0, count).
__device__ bool huf_stream(const ZTables& T, int maxb, const uint8_t* src, int32_t n, uint8_t* out, int32_t count) {
  BitB b;
  if (!b.init(src, n)) return false;
  for (int32_t i = 0; i < count; ++i) {
    if (b.used + maxb > 64) b.reload();
    const uint32_t e = T.huf[b.peek(maxb)];
    out[i] = (uint8_t)(e & 0xff);
    b.used += (int32_t)(e >> 8);
    if (b.left() < 0) return false;
  }
  return b.left() == 0;
}

__device__ __forceinline__ uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t rd24(const uint8_t* p) { return rd16(p) | ((uint32_t)p[2] << 16); }
__device__ __forceinline__ uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }

struct FrameState {
  uint32_t rep0, rep1, rep2;
  int llog, olog, mlog;
  bool llv, olv, mlv, hufv;
  int hufbits;
};

// Optional per-frame phase counters (tools/zstd_bench.py): cycles in the Huffman table build, the literal streams,
// the sequence-table builds and the sequence loop, plus the frame's block / sequence / literal counts.
enum { P_TOTAL, P_HUFTAB, P_LITS, P_SEQTAB, P_SEQ, P_NBLK, P_NSEQ, P_NLIT, P_N };
struct Prof {
  int64_t v[P_N];
  bool on;
  __device__ __forceinline__ static int64_t now() { return (int64_t)__builtin_readcyclecounter(); }
};

// One compressed block at in[0, n) → out[op, ...); returns Z_OK and advances op, or an error.  `done`: output known
// complete (visible to every lane) at the last wait.
// Literal-length / match-length codes → base | extra bits << 24, staged in LDS per workgroup: the sequence loop's
// lookups are indexed by decoded values, and from __constant__ memory each would be a dependent global load.
struct CodeTabs {
  uint32_t ll[36];
  uint32_t ml[53];
};

__device__ int32_t decode_block(const uint8_t* in, int32_t n, uint8_t* out, int32_t& op, int32_t cap,
                                ZTables& T, const CodeTabs& C, FrameState& fs, int gl, int32_t& done, Prof& pf) {
  int64_t t0 = pf.on ? Prof::now() : 0;
  if (n < 1) return Z_TRUNC;
  const uint32_t b0 = in[0];
  const int lt = (int)(b0 & 3), sf = (int)((b0 >> 2) & 3);
  int32_t regen = 0, csize = 0, hdr = 0;
  int streams = 1;
  if (lt <= 1) {
    if (sf == 0 || sf == 2) { hdr = 1; regen = (int32_t)(b0 >> 3); }
    else if (sf == 1) { if (n < 2) return Z_TRUNC; hdr = 2; regen = (int32_t)((b0 >> 4) | ((uint32_t)in[1] << 4)); }
    else {
      if (n < 3) return Z_TRUNC;
      hdr = 3;
      regen = (int32_t)((b0 >> 4) | ((uint32_t)in[1] << 4) | ((uint32_t)in[2] << 12));
    }
    csize = lt == 0 ? regen : 1;
  } else if (sf <= 1) {
    if (n < 3) return Z_TRUNC;
    hdr = 3;
    const uint32_t h = rd24(in);
    regen = (int32_t)((h >> 4) & 0x3FF);
    csize = (int32_t)((h >> 14) & 0x3FF);
    streams = sf == 0 ? 1 : 4;
  } else if (sf == 2) {
    if (n < 4) return Z_TRUNC;
    hdr = 4;
    const uint32_t h = rd32(in);
    regen = (int32_t)((h >> 4) & 0x3FFF);
    csize = (int32_t)((h >> 18) & 0x3FFF);
    streams = 4;
  } else {
    if (n < 5) return Z_TRUNC;
    hdr = 5;
    const uint64_t h = (uint64_t)rd32(in) | ((uint64_t)in[4] << 32);
    regen = (int32_t)((h >> 4) & 0x3FFFF);
    csize = (int32_t)((h >> 22) & 0x3FFFF);
    streams = 4;
  }
  if (regen > kBlockMax || hdr + csize > n || regen > cap - op) return Z_LIT;
  // literal source: the input (raw), a byte (RLE), or the slot tail (Huffman)
  const uint8_t* lit = in + hdr;
  uint32_t rle = 0;
  if (lt == 1) rle = in[hdr];
  if (lt >= 2) {
    int32_t tree = 0;
    if (lt == 2) {
      int mb = 0;
      tree = read_huffman(in + hdr, csize, T, gl, &mb);
      if (tree < 0) return Z_HUF;
      fs.hufv = true;
      fs.hufbits = mb;
    } else if (!fs.hufv) {
      return Z_HUF;
    }
    if (pf.on) { const int64_t t = Prof::now(); pf.v[P_HUFTAB] += t - t0; t0 = t; pf.v[P_NLIT] += regen; }
    uint8_t* lbuf = out + (cap - regen);
    const uint8_t* sp = in + hdr + tree;
    const int32_t sn = csize - tree;
    bool ok = true;
    if (streams == 1) {
      if (gl == 0) ok = huf_stream(T, fs.hufbits, sp, sn, lbuf, regen);
    } else {
      if (sn < 6) return Z_LIT;
      const int32_t s1 = (int32_t)rd16(sp), s2 = (int32_t)rd16(sp + 2), s3 = (int32_t)rd16(sp + 4);
      const int32_t s4 = sn - 6 - s1 - s2 - s3;
      const int32_t per = (regen + 3) / 4;
      const int32_t last = regen - 3 * per;
      if (s4 < 1 || last < 0) return Z_LIT;
      if (gl < 4) {
        const int32_t off = gl == 0 ? 0 : gl == 1 ? s1 : gl == 2 ? s1 + s2 : s1 + s2 + s3;
        const int32_t len = gl == 0 ? s1 : gl == 1 ? s2 : gl == 2 ? s3 : s4;
        ok = huf_stream(T, fs.hufbits, sp + 6 + off, len, lbuf + gl * per, gl < 3 ? per : last);
      }
    }
    // every lane learns whether any stream failed; the literals become visible to the group
    const uint64_t bad = __ballot(!ok);
    const int grp = (int)((threadIdx.x & 63) & ~(ZG - 1));
    if ((bad >> grp) & kGroupMask) return Z_HUF;
    stores_visible();
    lit = lbuf;
    if (pf.on) { const int64_t t = Prof::now(); pf.v[P_LITS] += t - t0; t0 = t; }
  }
  // ---- sequences
  const uint8_t* sp = in + hdr + csize;
  const int32_t sn = n - hdr - csize;
  if (sn < 1) return Z_TRUNC;
  int32_t nseq, h2;
  if (sp[0] < 128) { nseq = sp[0]; h2 = 1; }
  else if (sp[0] < 255) { if (sn < 2) return Z_TRUNC; nseq = ((int32_t)(sp[0] - 128) << 8) + sp[1]; h2 = 2; }
  else { if (sn < 3) return Z_TRUNC; nseq = (int32_t)sp[1] + ((int32_t)sp[2] << 8) + 0x7F00; h2 = 3; }
  int32_t lpos = 0;
  // a literal run: from the input / slot tail, or a fill
  auto put_lits = [&](int32_t len) {
    for (int32_t c = gl; c < len; c += ZG) out[op + c] = lt == 1 ? (uint8_t)rle : lit[lpos + c];
  };
  if (nseq > 0) {
    if (sn < h2 + 1) return Z_TRUNC;
    const uint32_t modes = sp[h2];
    if (modes & 3) return Z_SEQ;
    int32_t q = h2 + 1, d;
    if ((d = seq_table((int)(modes >> 6), sp + q, sn - q, kLLDef, 36, 6, 9, 35, T, T.ll, &fs.llog, &fs.llv)) < 0)
      return Z_FSE;
    q += d;
    if ((d = seq_table((int)((modes >> 4) & 3), sp + q, sn - q, kOFDef, 29, 5, 8, 31, T, T.of, &fs.olog, &fs.olv))
        < 0)
      return Z_FSE;
    q += d;
    if ((d = seq_table((int)((modes >> 2) & 3), sp + q, sn - q, kMLDef, 53, 6, 9, 52, T, T.ml, &fs.mlog, &fs.mlv))
        < 0)
      return Z_FSE;
    q += d;
    if (pf.on) { const int64_t t = Prof::now(); pf.v[P_SEQTAB] += t - t0; t0 = t; pf.v[P_NSEQ] += nseq; }
    BitB b;
    if (!b.init(sp + q, sn - q)) return Z_SEQ;
    uint32_t sll = b.read(fs.llog), sof = b.read(fs.olog), sml = b.read(fs.mlog);
    for (int32_t i = 0; i < nseq; ++i) {
      const uint32_t el = T.ll[sll], eo = T.of[sof], em = T.ml[sml];
      const uint32_t llc = (el >> 8) & 0xff, ofc = (eo >> 8) & 0xff, mlc = (em >> 8) & 0xff;
      if (llc > 35 || mlc > 52 || ofc > 31) return Z_SEQ;
      uint32_t ofv;
      if (ofc > 24) {                       // > 24 extra bits: read in two parts (the container holds 64)
        const uint32_t hi = b.read((int)ofc - 24);
        ofv = (1u << ofc) + (hi << 24) + b.read(24);
      } else {
        ofv = (1u << ofc) + b.read((int)ofc);
      }
      const uint32_t cm = C.ml[mlc], cl = C.ll[llc];
      const int32_t ml = (int32_t)((cm & 0xFFFFFFu) + b.read((int)(cm >> 24)));
      const int32_t ll = (int32_t)((cl & 0xFFFFFFu) + b.read((int)(cl >> 24)));
      uint32_t off;
      if (ofv > 3) {
        off = ofv - 3;
        fs.rep2 = fs.rep1;
        fs.rep1 = fs.rep0;
        fs.rep0 = off;
      } else {
        const int idx = (int)ofv - 1 + (ll == 0 ? 1 : 0);
        if (idx == 0) {
          off = fs.rep0;
        } else {
          off = idx == 3 ? fs.rep0 - 1 : (idx == 1 ? fs.rep1 : fs.rep2);
          if (idx > 1) fs.rep2 = fs.rep1;
          fs.rep1 = fs.rep0;
          fs.rep0 = off;
        }
      }
      if (i + 1 < nseq) {                   // state updates: literal lengths, match lengths, offsets
        sll = (el >> 16) + b.read((int)(el & 0xff));
        sml = (em >> 16) + b.read((int)(em & 0xff));
        sof = (eo >> 16) + b.read((int)(eo & 0xff));
      }
      if (b.left() < 0) return Z_SEQ;
      if (ll > regen - lpos || ll > cap - op || ml > cap - op - ll) return Z_OVERFLOW;
      put_lits(ll);
      op += ll;
      lpos += ll;
      if (off == 0 || (int32_t)off > op) return Z_OFFSET;
      const int32_t s = op - (int32_t)off;
      if (s + (ml < (int32_t)off ? ml : (int32_t)off) > done) {   // source reaches past the visible output
        stores_visible();
        done = op;
      }
      for (int32_t c = gl; c < ml; c += ZG) out[op + c] = out[s + (c < (int32_t)off ? c : c % (int32_t)off)];
      op += ml;
    }
    if (b.left() != 0) return Z_SEQ;
    if (pf.on) pf.v[P_SEQ] += Prof::now() - t0;
  }
  const int32_t rest = regen - lpos;
  if (rest > cap - op) return Z_OVERFLOW;
  put_lits(rest);
  op += rest;
  return Z_OK;
}

__global__ __launch_bounds__(ZWG) void zstd_frame_kernel(const uint8_t* __restrict__ src,
                                                          const int64_t* __restrict__ comp_off,
                                                          const int32_t* __restrict__ comp_len,
                                                          const uint8_t* __restrict__ kind,
                                                          const int64_t* __restrict__ out_off,
                                                          const int64_t* __restrict__ cap_arr, int64_t nb,
                                                          uint8_t* __restrict__ dst, int64_t* __restrict__ produced,
                                                          int32_t* __restrict__ status, int64_t* __restrict__ prof) {
  __shared__ ZTables tabs[ZWG / ZG];
  __shared__ CodeTabs codes;
  ZTables& T = tabs[threadIdx.x / ZG];
  for (int k = threadIdx.x; k < 36 + 53; k += ZWG) {       // (whole workgroup, before any early exit)
    if (k < 36) codes.ll[k] = kLLBase[k] | ((uint32_t)kLLBits[k] << 24);
    else codes.ml[k - 36] = kMLBase[k - 36] | ((uint32_t)kMLBits[k - 36] << 24);
  }
  __syncthreads();
  const int64_t b = ((int64_t)blockIdx.x * ZWG + threadIdx.x) / ZG;
  const int gl = (int)(threadIdx.x & (ZG - 1));
  if (b >= nb || kind[b] != 4) return;
  const uint8_t* in = src + comp_off[b];
  const int32_t n = comp_len[b];
  const int64_t cap64 = cap_arr[b];
  uint8_t* out = dst + out_off[b];
  int32_t rc = Z_OK;
  int32_t op = 0;
  if (n < 6 || cap64 < 0 || cap64 > INT32_MAX) rc = Z_HEADER;
  const int32_t cap = (int32_t)cap64;
  int32_t ip = 0;
  int32_t bmax = kBlockMax;
  bool checksum = false;
  int64_t fcs = -1;
  if (rc == Z_OK) {
    if (rd32(in) != 0xFD2FB528u) rc = Z_HEADER;
    const uint32_t fhd = in[4];
    const int fcs_flag = (int)(fhd >> 6);
    const bool single = (fhd >> 5) & 1;
    const int did_flag = (int)(fhd & 3);
    checksum = (fhd >> 2) & 1;
    if ((fhd >> 3) & 1) rc = Z_HEADER;
    ip = 5;
    int64_t window = 0;
    if (!single) {
      const uint32_t wd = in[ip++];
      const int64_t base = (int64_t)1 << (10 + (wd >> 3));
      window = base + (base / 8) * (wd & 7);
    }
    const int did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    for (int k = 0; k < did_len; ++k)
      if (ip + k < n && in[ip + k]) rc = Z_HEADER;                       // dictionaries: not supported
    ip += did_len;
    const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (ip + fcs_len > n) rc = Z_TRUNC;
    if (rc == Z_OK) {
      if (fcs_len == 1) fcs = in[ip];
      else if (fcs_len == 2) fcs = (int64_t)rd16(in + ip) + 256;
      else if (fcs_len == 4) fcs = rd32(in + ip);
      else if (fcs_len == 8) fcs = (int64_t)rd32(in + ip) | ((int64_t)rd32(in + ip + 4) << 32);
    }
    ip += fcs_len;
    if (single) window = fcs;
    if (window > 0 && window < bmax) bmax = (int32_t)window;
  }
  Prof pf;
  pf.on = prof != nullptr;
  for (int k = 0; k < P_N; ++k) pf.v[k] = 0;
  const int64_t tf = pf.on ? Prof::now() : 0;
  FrameState fs;
  fs.rep0 = 1; fs.rep1 = 4; fs.rep2 = 8;
  fs.llog = fs.olog = fs.mlog = 0;
  fs.llv = fs.olv = fs.mlv = fs.hufv = false;
  fs.hufbits = 0;
  int32_t done = 0;
  while (rc == Z_OK) {
    if (ip + 3 > n) { rc = Z_TRUNC; break; }
    const uint32_t bh = rd24(in + ip);
    const bool last = bh & 1;
    const int type = (int)((bh >> 1) & 3);
    const int32_t size = (int32_t)(bh >> 3);
    ip += 3;
    if (type == 0) {
      if (ip + size > n) { rc = Z_TRUNC; break; }
      if (size > cap - op) { rc = Z_OVERFLOW; break; }
      for (int32_t c = gl; c < size; c += ZG) out[op + c] = in[ip + c];
      op += size;
      ip += size;
    } else if (type == 1) {
      if (ip + 1 > n) { rc = Z_TRUNC; break; }
      if (size > cap - op) { rc = Z_OVERFLOW; break; }
      const uint8_t v = in[ip];
      for (int32_t c = gl; c < size; c += ZG) out[op + c] = v;
      op += size;
      ip += 1;
    } else if (type == 2) {
      if (size > bmax || ip + size > n) { rc = Z_BLOCK; break; }
      const int32_t op0 = op;
      rc = decode_block(in + ip, size, out, op, cap, T, codes, fs, gl, done, pf);
      ++pf.v[P_NBLK];
      if (rc == Z_OK && op - op0 > bmax) rc = Z_BLOCK;
      ip += size;
    } else {
      rc = Z_BLOCK;
    }
    if (last) break;
  }
  if (rc == Z_OK && checksum) ip += 4;
  if (rc == Z_OK && ip > n) rc = Z_TRUNC;
  if (rc == Z_OK && fcs >= 0 && op != fcs) rc = Z_SIZE;
  if (gl == 0) {
    status[b] = rc;
    produced[b] = rc == Z_OK ? op : 0;
    if (pf.on) {
      pf.v[P_TOTAL] = Prof::now() - tf;
      for (int k = 0; k < P_N; ++k) prof[b * P_N + k] = pf.v[k];
    }
  }
}

}  // namespace

// Decode every kind-4 (zstd frame) entry of a block table into its capacity slot; other kinds are left alone (the
// LZ4 / deflate / snappy kernels take them).  produced[b] = the frame's decoded size.
DXA_API int dxa_zstd_decode_into(const void* src, const void* comp_off, const void* comp_len, const void* kind,
                                 const void* out_off, const void* cap, int64_t nb, void* dst, void* produced,
                                 void* status, void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(zstd_frame_kernel, dim3((unsigned)((nb * ZG + ZWG - 1) / ZWG)), dim3(ZWG), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)kind,
                     (const int64_t*)out_off, (const int64_t*)cap, nb, (uint8_t*)dst, (int64_t*)produced,
                     (int32_t*)status, (int64_t*)nullptr);
  return (int)hipGetLastError();
}

// The same decode with per-frame phase counters: prof[b * 8 + k] (k: total / Huffman table / literal streams /
// sequence tables / sequence loop cycles, blocks, sequences, literals).  Measurement tool only.
DXA_API int dxa_zstd_decode_prof(const void* src, const void* comp_off, const void* comp_len, const void* kind,
                                 const void* out_off, const void* cap, int64_t nb, void* dst, void* produced,
                                 void* status, void* prof, void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(zstd_frame_kernel, dim3((unsigned)((nb * ZG + ZWG - 1) / ZWG)), dim3(ZWG), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)kind,
                     (const int64_t*)out_off, (const int64_t*)cap, nb, (uint8_t*)dst, (int64_t*)produced,
                     (int32_t*)status, (int64_t*)prof);
  return (int)hipGetLastError();
}
