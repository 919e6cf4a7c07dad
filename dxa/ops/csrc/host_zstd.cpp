// Zstandard decoder (host reference), written from RFC 8878; see dxa_zstd.h.  Straightforward and checked at
// every step — it is the oracle the device decoder (zstd.hip) is tested against, and the host fallback of the Kafka
// codec-4 source.  Also exports a compressor entry point that forwards to the system libzstd when it is present
// (dlopen at run time; used only to produce test / benchmark batches, as a Kafka producer would).
#include "dxa_zstd.h"

#include <dlfcn.h>

#include <cstring>
#include <vector>

namespace dxa {
namespace zstd {
namespace {

enum : int64_t {
  kErrTrunc = -1, kErrDict = -2, kErrMagic = -3, kErrBlock = -4, kErrLiterals = -5, kErrHuffman = -6,
  kErrFse = -7, kErrSeq = -8, kErrOffset = -9, kErrOverflow = -10, kErrReserved = -11
};

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr int64_t kBlockMax = 128 * 1024;

inline uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
inline uint32_t le24(const uint8_t* p) { return le16(p) | ((uint32_t)p[2] << 16); }
inline uint32_t le32(const uint8_t* p) { return le16(p) | (le16(p + 2) << 16); }
inline uint64_t le64(const uint8_t* p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }
inline int highbit(uint32_t v) { return 31 - __builtin_clz(v); }

// ---- bit readers ----------------------------------------------------------------------------------------------
// Forward (FSE table descriptions): little-endian bit order from the start.
struct FwdBits {
  const uint8_t* p;
  int64_t n;
  int64_t bit = 0;
  uint32_t peek(int k) const {
    uint32_t v = 0;
    for (int i = 0; i < k; ++i) {
      const int64_t b = bit + i;
      const uint32_t x = b / 8 < n ? (p[b / 8] >> (b % 8)) & 1u : 0u;
      v |= x << i;
    }
    return v;
  }
  void skip(int k) { bit += k; }
  uint32_t read(int k) {
    const uint32_t v = peek(k);
    skip(k);
    return v;
  }
};

// Backward (Huffman streams, FSE bitstreams): starts below the final marker bit and reads towards byte 0; bits
// wanted below position 0 read as zeros and leave `pos` negative (the overflow the decoders test).
struct BackBits {
  const uint8_t* p;
  int64_t pos;                  // bits remaining
  bool init(const uint8_t* src, int64_t n) {
    p = src;
    if (n <= 0 || src[n - 1] == 0) return false;
    pos = n * 8 - (8 - highbit(src[n - 1]));
    return true;
  }
  uint64_t read(int k) {
    if (k == 0) return 0;
    pos -= k;
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) {
      const int64_t b = pos + i;
      const uint64_t x = b >= 0 ? (p[b / 8] >> (b % 8)) & 1u : 0u;
      v |= x << i;
    }
    return v;
  }
  uint64_t peek(int k) const {
    BackBits c = *this;
    return c.read(k);
  }
};

// ---- FSE ------------------------------------------------------------------------------------------------------
struct FseCell {
  uint16_t base;
  uint8_t sym;
  uint8_t bits;
};

struct FseTable {
  int log = 0;
  std::vector<FseCell> cells;
  bool valid = false;
};

bool fse_build(const int16_t* norm, int nsym, int log, FseTable& t) {
  const int size = 1 << log;
  t.log = log;
  t.cells.assign((size_t)size, FseCell{0, 0, 0});
  std::vector<uint32_t> next((size_t)nsym);
  int high = size - 1;
  for (int s = 0; s < nsym; ++s) {
    if (norm[s] == -1) {
      t.cells[(size_t)high--].sym = (uint8_t)s;
      next[(size_t)s] = 1;
    } else {
      next[(size_t)s] = (uint32_t)norm[s];
    }
  }
  const int step = (size >> 1) + (size >> 3) + 3;
  int pos = 0;
  for (int s = 0; s < nsym; ++s) {
    for (int i = 0; i < norm[s]; ++i) {
      t.cells[(size_t)pos].sym = (uint8_t)s;
      do { pos = (pos + step) & (size - 1); } while (pos > high);
    }
  }
  if (pos != 0) return false;
  for (int c = 0; c < size; ++c) {
    const int s = t.cells[(size_t)c].sym;
    const uint32_t x = next[(size_t)s]++;
    if (x == 0) return false;
    const int nb = log - highbit(x);
    t.cells[(size_t)c].bits = (uint8_t)nb;
    t.cells[(size_t)c].base = (uint16_t)((x << nb) - (uint32_t)size);
  }
  t.valid = true;
  return true;
}

// FSE table description (RFC 8878 4.1.1) at src → normalized counts; returns bytes consumed or -1.
int64_t fse_read_counts(const uint8_t* src, int64_t n, int max_log, int max_sym, int16_t* norm, int* nsym, int* log) {
  FwdBits r{src, n};
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
      while (r.peek(16) == 0xFFFF) { n0 += 24; r.skip(16); }
      while ((r.peek(2) & 3) == 3) { n0 += 3; r.skip(2); }
      n0 += (int)r.read(2);
      if (n0 > max_sym + 1) return -1;
      while (s < n0) norm[s++] = 0;
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
    norm[s++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
  }
  if (remaining != 1 || s > max_sym + 1) return -1;
  *nsym = s;
  *log = al;
  const int64_t used = (r.bit + 7) / 8;
  return used <= n ? used : -1;
}

// ---- Huffman --------------------------------------------------------------------------------------------------
struct HufTable {
  int max_bits = 0;
  std::vector<uint8_t> sym, bits;       // 2^max_bits entries
  bool valid = false;
};

// Huffman tree description → decode table; returns bytes consumed or an error.
int64_t huf_read(const uint8_t* src, int64_t n, HufTable& h) {
  if (n < 1) return kErrTrunc;
  uint8_t w[256];
  int nw = 0;
  int64_t used;
  const int hb = src[0];
  if (hb < 128) {
    // FSE-compressed weights: a table description (accuracy <= 6), then two interleaved states on one backward
    // bitstream, decoded until it overflows
    if (hb + 1 > n) return kErrTrunc;
    int16_t norm[256];
    int nsym = 0, log = 0;
    const int64_t d = fse_read_counts(src + 1, hb, 6, 255, norm, &nsym, &log);
    if (d < 0) return kErrHuffman;
    FseTable t;
    if (!fse_build(norm, nsym, log, t)) return kErrHuffman;
    BackBits b;
    if (!b.init(src + 1 + d, hb - d)) return kErrHuffman;
    uint32_t s1 = (uint32_t)b.read(log), s2 = (uint32_t)b.read(log);
    while (true) {
      if (nw + 2 > 255) return kErrHuffman;
      w[nw++] = t.cells[s1].sym;
      s1 = t.cells[s1].base + (uint32_t)b.read(t.cells[s1].bits);
      if (b.pos < 0) { w[nw++] = t.cells[s2].sym; break; }
      w[nw++] = t.cells[s2].sym;
      s2 = t.cells[s2].base + (uint32_t)b.read(t.cells[s2].bits);
      if (b.pos < 0) { w[nw++] = t.cells[s1].sym; break; }
    }
    used = 1 + hb;
  } else {
    nw = hb - 127;
    const int64_t bytes = (nw + 1) / 2;
    if (1 + bytes > n) return kErrTrunc;
    for (int i = 0; i < nw; ++i) {
      const uint8_t x = src[1 + i / 2];
      w[i] = (i & 1) ? (x & 15) : (x >> 4);
    }
    used = 1 + bytes;
  }
  // the last symbol's weight completes the sum of 2^(w-1) to a power of two
  uint32_t sum = 0;
  for (int i = 0; i < nw; ++i) {
    if (w[i] > 11) return kErrHuffman;
    if (w[i]) sum += 1u << (w[i] - 1);
  }
  if (sum == 0) return kErrHuffman;
  const int maxb = highbit(sum) + 1;
  if (maxb > 11) return kErrHuffman;
  const uint32_t rest = (1u << maxb) - sum;
  if (rest & (rest - 1)) return kErrHuffman;
  w[nw++] = (uint8_t)(highbit(rest) + 1);
  h.max_bits = maxb;
  h.sym.assign((size_t)1 << maxb, 0);
  h.bits.assign((size_t)1 << maxb, 0);
  // symbols of weight k occupy 2^(k-1) consecutive entries each; weights ascending, then symbol order
  uint32_t start[13] = {0};
  uint32_t cnt[13] = {0};
  for (int i = 0; i < nw; ++i) ++cnt[w[i]];
  uint32_t pos = 0;
  for (int k = 1; k <= maxb; ++k) {
    start[k] = pos;
    pos += cnt[k] << (k - 1);
  }
  if (pos != (1u << maxb)) return kErrHuffman;
  for (int i = 0; i < nw; ++i) {
    const int k = w[i];
    if (!k) continue;
    const uint32_t len = 1u << (k - 1);
    for (uint32_t j = 0; j < len; ++j) {
      h.sym[start[k] + j] = (uint8_t)i;
      h.bits[start[k] + j] = (uint8_t)(maxb + 1 - k);
    }
    start[k] += len;
  }
  h.valid = true;
  return used;
}

bool huf_stream(const HufTable& h, const uint8_t* src, int64_t n, uint8_t* out, int64_t count) {
  BackBits b;
  if (!b.init(src, n)) return false;
  for (int64_t i = 0; i < count; ++i) {
    const uint32_t idx = (uint32_t)b.peek(h.max_bits);
    out[i] = h.sym[idx];
    b.read(h.bits[idx]);
    if (b.pos < 0) return false;
  }
  return b.pos == 0;
}

// ---- sequences ------------------------------------------------------------------------------------------------
const int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2,
                                2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
const int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
const int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                -1, -1, -1, -1, -1};
const uint32_t kLLBase[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32, 40,
                              48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                             4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const uint32_t kMLBase[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                              26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131,
                              259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

struct FrameState {
  HufTable huf;
  FseTable ll, of, ml;
  uint32_t rep[3] = {1, 4, 8};
};

// Table of one sequence symbol kind by mode; returns bytes consumed or an error.
int64_t seq_table(int mode, const uint8_t* src, int64_t n, const int16_t* def, int def_n, int def_log, int max_log,
                  int max_sym, FseTable& t) {
  if (mode == 0) {
    if (!fse_build(def, def_n, def_log, t)) return kErrFse;
    return 0;
  }
  if (mode == 1) {                              // RLE: one symbol, no state bits
    if (n < 1 || src[0] > max_sym) return kErrFse;
    t.log = 0;
    t.cells.assign(1, FseCell{0, src[0], 0});
    t.valid = true;
    return 1;
  }
  if (mode == 2) {
    int16_t norm[64];
    int nsym = 0, log = 0;
    const int64_t d = fse_read_counts(src, n, max_log, max_sym, norm, &nsym, &log);
    if (d < 0 || !fse_build(norm, nsym, log, t)) return kErrFse;
    return d;
  }
  return t.valid ? 0 : kErrFse;                 // repeat: the previous block's table
}

int64_t decode_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t op0, int64_t cap, FrameState& fs,
                     int64_t block_max, int64_t frame0) {
  // ---- literals
  if (n < 1) return kErrTrunc;
  const int lt = src[0] & 3;
  const int sf = (src[0] >> 2) & 3;
  int64_t regen = 0, csize = 0, hdr = 0;
  int streams = 1;
  if (lt <= 1) {
    if (sf == 0 || sf == 2) { hdr = 1; regen = src[0] >> 3; }
    else if (sf == 1) { if (n < 2) return kErrTrunc; hdr = 2; regen = (src[0] >> 4) | ((int64_t)src[1] << 4); }
    else { if (n < 3) return kErrTrunc; hdr = 3; regen = (src[0] >> 4) | ((int64_t)src[1] << 4) | ((int64_t)src[2] << 12); }
    csize = lt == 0 ? regen : 1;
  } else {
    if (sf <= 1) {
      if (n < 3) return kErrTrunc;
      hdr = 3;
      const uint32_t h = le24(src);
      regen = (h >> 4) & 0x3FF;
      csize = (h >> 14) & 0x3FF;
      streams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (n < 4) return kErrTrunc;
      hdr = 4;
      const uint32_t h = le32(src);
      regen = (h >> 4) & 0x3FFF;
      csize = (h >> 18) & 0x3FFF;
      streams = 4;
    } else {
      if (n < 5) return kErrTrunc;
      hdr = 5;
      const uint64_t h = (uint64_t)le32(src) | ((uint64_t)src[4] << 32);
      regen = (int64_t)((h >> 4) & 0x3FFFF);
      csize = (int64_t)((h >> 22) & 0x3FFFF);
      streams = 4;
    }
  }
  if (regen > block_max || hdr + csize > n) return kErrLiterals;
  std::vector<uint8_t> lit((size_t)regen + 8);
  const uint8_t* lp = src + hdr;
  if (lt == 0) {
    std::memcpy(lit.data(), lp, (size_t)regen);
  } else if (lt == 1) {
    std::memset(lit.data(), lp[0], (size_t)regen);
  } else {
    int64_t tree = 0;
    if (lt == 2) {
      tree = huf_read(lp, csize, fs.huf);
      if (tree < 0) return tree;
    } else if (!fs.huf.valid) {
      return kErrHuffman;
    }
    const uint8_t* sp = lp + tree;
    const int64_t sn = csize - tree;
    if (streams == 1) {
      if (!huf_stream(fs.huf, sp, sn, lit.data(), regen)) return kErrHuffman;
    } else {
      if (sn < 6) return kErrLiterals;
      const int64_t s1 = le16(sp), s2 = le16(sp + 2), s3 = le16(sp + 4);
      const int64_t s4 = sn - 6 - s1 - s2 - s3;
      if (s4 < 1) return kErrLiterals;
      const int64_t per = (regen + 3) / 4;
      const int64_t last = regen - 3 * per;
      if (last < 0) return kErrLiterals;
      const uint8_t* q = sp + 6;
      const int64_t sz[4] = {s1, s2, s3, s4};
      for (int k = 0; k < 4; ++k) {
        if (!huf_stream(fs.huf, q, sz[k], lit.data() + k * per, k < 3 ? per : last)) return kErrHuffman;
        q += sz[k];
      }
    }
  }
  // ---- sequences
  const uint8_t* sp = src + hdr + csize;
  int64_t sn = n - hdr - csize;
  if (sn < 1) return kErrTrunc;
  int64_t nseq;
  int64_t h2;
  if (sp[0] < 128) { nseq = sp[0]; h2 = 1; }
  else if (sp[0] < 255) { if (sn < 2) return kErrTrunc; nseq = ((int64_t)(sp[0] - 128) << 8) + sp[1]; h2 = 2; }
  else { if (sn < 3) return kErrTrunc; nseq = (int64_t)sp[1] + ((int64_t)sp[2] << 8) + 0x7F00; h2 = 3; }
  int64_t op = op0;
  int64_t lpos = 0;
  if (nseq > 0) {
    if (sn < h2 + 1) return kErrTrunc;
    const uint8_t modes = sp[h2];
    if (modes & 3) return kErrReserved;
    int64_t q = h2 + 1;
    int64_t d;
    if ((d = seq_table(modes >> 6, sp + q, sn - q, kLLDefault, 36, 6, 9, 35, fs.ll)) < 0) return d;
    q += d;
    if ((d = seq_table((modes >> 4) & 3, sp + q, sn - q, kOFDefault, 29, 5, 8, 31, fs.of)) < 0) return d;
    q += d;
    if ((d = seq_table((modes >> 2) & 3, sp + q, sn - q, kMLDefault, 53, 6, 9, 52, fs.ml)) < 0) return d;
    q += d;
    BackBits b;
    if (!b.init(sp + q, sn - q)) return kErrSeq;
    uint32_t sll = (uint32_t)b.read(fs.ll.log), sof = (uint32_t)b.read(fs.of.log), sml = (uint32_t)b.read(fs.ml.log);
    for (int64_t i = 0; i < nseq; ++i) {
      const int llc = fs.ll.cells[sll].sym, ofc = fs.of.cells[sof].sym, mlc = fs.ml.cells[sml].sym;
      if (llc > 35 || mlc > 52 || ofc > 31) return kErrSeq;
      const uint64_t ofv = (1ull << ofc) + b.read(ofc);
      const int64_t ml = kMLBase[mlc] + b.read(kMLBits[mlc]);
      const int64_t ll = kLLBase[llc] + b.read(kLLBits[llc]);
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        fs.rep[2] = fs.rep[1];
        fs.rep[1] = fs.rep[0];
        fs.rep[0] = (uint32_t)off;
      } else {
        const int idx = (int)ofv - 1 + (ll == 0 ? 1 : 0);
        if (idx == 0) {
          off = fs.rep[0];
        } else {
          off = idx == 3 ? (uint64_t)fs.rep[0] - 1 : fs.rep[idx];
          if (idx > 1) fs.rep[2] = fs.rep[1];
          fs.rep[1] = fs.rep[0];
          fs.rep[0] = (uint32_t)off;
        }
      }
      if (i + 1 < nseq) {                        // state updates: literal lengths, match lengths, offsets
        sll = fs.ll.cells[sll].base + (uint32_t)b.read(fs.ll.cells[sll].bits);
        sml = fs.ml.cells[sml].base + (uint32_t)b.read(fs.ml.cells[sml].bits);
        sof = fs.of.cells[sof].base + (uint32_t)b.read(fs.of.cells[sof].bits);
      }
      if (b.pos < 0) return kErrSeq;
      if (ll > regen - lpos || ll + ml > cap - op) return kErrOverflow;
      std::memcpy(dst + op, lit.data() + lpos, (size_t)ll);
      op += ll;
      lpos += ll;
      if (off == 0 || (int64_t)off > op - frame0) return kErrOffset;     // within this frame's output
      for (int64_t k = 0; k < ml; ++k) dst[op + k] = dst[op - (int64_t)off + k];
      op += ml;
    }
    if (b.pos != 0) return kErrSeq;
  }
  const int64_t rest = regen - lpos;
  if (rest > cap - op) return kErrOverflow;
  std::memcpy(dst + op, lit.data() + lpos, (size_t)rest);
  op += rest;
  if (op - op0 > block_max) return kErrBlock;
  return op - op0;
}

int64_t header(const uint8_t* src, int64_t n, FrameInfo* fi) {
  if (n < 4) return kErrTrunc;
  if (le32(src) != kMagic) return kErrMagic;
  if (n < 6) return kErrTrunc;
  const uint8_t fhd = src[4];
  const int fcs_flag = fhd >> 6;
  const bool single = (fhd >> 5) & 1;
  if ((fhd >> 3) & 1) return kErrReserved;
  const int did_flag = fhd & 3;
  int64_t p = 5;
  int64_t window = 0;
  if (!single) {
    const uint8_t wd = src[p++];
    const int exp = wd >> 3, man = wd & 7;
    const int64_t base = (int64_t)1 << (10 + exp);
    window = base + (base / 8) * man;
  }
  const int did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
  if (p + did_len > n) return kErrTrunc;
  uint32_t did = 0;
  for (int k = 0; k < did_len; ++k) did |= (uint32_t)src[p + k] << (8 * k);
  if (did) return kErrDict;
  p += did_len;
  const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
  if (p + fcs_len > n) return kErrTrunc;
  int64_t fcs = -1;
  if (fcs_len == 1) fcs = src[p];
  else if (fcs_len == 2) fcs = (int64_t)le16(src + p) + 256;
  else if (fcs_len == 4) fcs = le32(src + p);
  else if (fcs_len == 8) fcs = (int64_t)le64(src + p);
  p += fcs_len;
  if (single) window = fcs;
  fi->header_len = p;
  fi->content_size = fcs;
  fi->window = window;
  fi->checksum = (fhd >> 2) & 1;
  return 0;
}

}  // namespace

int frame_info(const uint8_t* src, int64_t n, FrameInfo* fi) {
  const int64_t rc = header(src, n, fi);
  if (rc == kErrDict) return -2;
  if (rc == kErrMagic) return -3;
  if (rc < 0) return -1;
  const int64_t bmax = fi->window < kBlockMax ? (fi->window > 0 ? fi->window : kBlockMax) : kBlockMax;
  int64_t p = fi->header_len;
  int32_t nb = 0;
  int64_t bound = 0;
  while (true) {
    if (p + 3 > n) return -1;
    const uint32_t bh = le24(src + p);
    const int last = bh & 1, type = (bh >> 1) & 3;
    const int64_t size = bh >> 3;
    if (type == 3) return -1;
    p += 3;
    const int64_t body = type == 1 ? 1 : size;
    if (size > bmax || p + body > n) return -1;            // RFC 8878 3.1.1.2.3: no block exceeds Block_Maximum_Size
    p += body;
    bound += type == 2 ? bmax : size;
    ++nb;
    if (last) break;
  }
  if (fi->checksum) p += 4;
  if (p > n) return -1;
  fi->end = p;
  fi->nblocks = nb;
  // the header's content size is untrusted: a frame can never decode to more than its blocks' maxima, so a larger
  // claim is a corrupt frame (and must not size an allocation)
  if (fi->content_size > bound) return -1;
  fi->bound = fi->content_size >= 0 ? fi->content_size : bound;
  return 0;
}

int64_t decompressed_bound(const uint8_t* src, int64_t n) {
  int64_t p = 0, total = 0;
  while (p < n) {
    if (n - p >= 8 && (le32(src + p) & 0xFFFFFFF0u) == 0x184D2A50u) {
      p += 8 + (int64_t)le32(src + p + 4);
      continue;
    }
    FrameInfo fi;
    if (frame_info(src + p, n - p, &fi) != 0) return -1;
    total += fi.bound;
    p += fi.end;
  }
  return total;
}

int64_t decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int64_t p = 0, op = 0;
  while (p < n) {
    if (n - p >= 8 && (le32(src + p) & 0xFFFFFFF0u) == 0x184D2A50u) {      // skippable frame
      const int64_t sz = le32(src + p + 4);
      if (p + 8 + sz > n) return kErrTrunc;
      p += 8 + sz;
      continue;
    }
    FrameInfo fi;
    const int64_t rc = header(src + p, n - p, &fi);
    if (rc < 0) return rc;
    const int64_t bmax = fi.window < kBlockMax ? (fi.window > 0 ? fi.window : kBlockMax) : kBlockMax;
    FrameState fs;
    const int64_t f0 = op;
    int64_t q = p + fi.header_len;
    while (true) {
      if (q + 3 > n) return kErrTrunc;
      const uint32_t bh = le24(src + q);
      const int last = bh & 1, type = (bh >> 1) & 3;
      const int64_t size = bh >> 3;
      q += 3;
      if (type == 3) return kErrReserved;
      if (type == 0) {
        if (q + size > n) return kErrTrunc;
        if (size > cap - op) return kErrOverflow;
        std::memcpy(dst + op, src + q, (size_t)size);
        op += size;
        q += size;
      } else if (type == 1) {
        if (q + 1 > n) return kErrTrunc;
        if (size > cap - op) return kErrOverflow;
        std::memset(dst + op, src[q], (size_t)size);
        op += size;
        q += 1;
      } else {
        if (size > bmax || q + size > n) return kErrBlock;
        const int64_t m = decode_block(src + q, size, dst, op, cap, fs, bmax, f0);
        if (m < 0) return m;
        op += m;
        q += size;
      }
      if (last) break;
    }
    if (fi.checksum) q += 4;
    if (q > n) return kErrTrunc;
    if (fi.content_size >= 0 && op - f0 != fi.content_size) return kErrBlock;
    p = q;
  }
  return op;
}

}  // namespace zstd
}  // namespace dxa

namespace {
typedef size_t (*zstd_bound_fn)(size_t);
typedef unsigned (*zstd_iserror_fn)(size_t);
typedef void* (*zstd_create_fn)();
typedef size_t (*zstd_free_fn)(void*);
typedef size_t (*zstd_setp_fn)(void*, int, int);
typedef size_t (*zstd_compress2_fn)(void*, void*, size_t, const void*, size_t);

// the system libzstd, resolved at run time (no build dependency): ZSTD_compress2 with explicit frame parameters
struct LibZstd {
  zstd_bound_fn bound = nullptr;
  zstd_iserror_fn is_error = nullptr;
  zstd_create_fn create = nullptr;
  zstd_free_fn free_ctx = nullptr;
  zstd_setp_fn set_param = nullptr;
  zstd_compress2_fn compress2 = nullptr;
  LibZstd() {
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    bound = (zstd_bound_fn)dlsym(h, "ZSTD_compressBound");
    is_error = (zstd_iserror_fn)dlsym(h, "ZSTD_isError");
    create = (zstd_create_fn)dlsym(h, "ZSTD_createCCtx");
    free_ctx = (zstd_free_fn)dlsym(h, "ZSTD_freeCCtx");
    set_param = (zstd_setp_fn)dlsym(h, "ZSTD_CCtx_setParameter");
    compress2 = (zstd_compress2_fn)dlsym(h, "ZSTD_compress2");
  }
  bool ok() const { return bound && is_error && create && free_ctx && set_param && compress2; }
};
const LibZstd& libzstd() {
  static LibZstd z;
  return z;
}
constexpr int kParamLevel = 100, kParamContentSize = 200, kParamChecksum = 201;    // ZSTD_cParameter values
}  // namespace

extern "C" {

__attribute__((visibility("default"))) int64_t dxa_zstd_decompress(const uint8_t* src, int64_t n, uint8_t* dst,
                                                                   int64_t cap) {
  return dxa::zstd::decompress(src, n, dst, cap);
}

__attribute__((visibility("default"))) int64_t dxa_zstd_bound(const uint8_t* src, int64_t n) {
  return dxa::zstd::decompressed_bound(src, n);
}

// Producer side (tests, simulated producers): one frame from the system libzstd.  flags bit 0: write the content
// size (zstd-jni's streaming ZstdOutputStream, which Kafka uses, does not), bit 1: append the XXH64 checksum.
// Returns -1 when libzstd is not installed, -2 on a compression error.
__attribute__((visibility("default"))) int64_t dxa_zstd_compress(const uint8_t* src, int64_t n, uint8_t* dst,
                                                                 int64_t cap, int32_t level, int32_t flags) {
  const LibZstd& z = libzstd();
  if (!z.ok()) return -1;
  void* c = z.create();
  if (!c) return -2;
  z.set_param(c, kParamLevel, level);
  z.set_param(c, kParamContentSize, flags & 1);
  z.set_param(c, kParamChecksum, (flags >> 1) & 1);
  const size_t r = z.compress2(c, dst, (size_t)cap, src, (size_t)n);
  z.free_ctx(c);
  if (z.is_error(r)) return -2;
  return (int64_t)r;
}

__attribute__((visibility("default"))) int64_t dxa_zstd_compress_bound(int64_t n) {
  const LibZstd& z = libzstd();
  return z.bound ? (int64_t)z.bound((size_t)n) : -1;
}

}  // extern "C"
