// Kafka record-batch (message format v2) codec for the ingest path — native so a 1 M events/s source does not pay
// Python per record.  Decoding turns the raw bytes of a Fetch response's record set into one contiguous, 16-byte
// padded value buffer + offsets (exactly what the GPU JSON parser consumes after one H2D copy).  Encoding builds
// an uncompressed v2 batch for the producer.  CRC-32C (Castagnoli) is slicing-by-8.
//
// Record batch v2:
//   baseOffset i64 | batchLength i32 | partitionLeaderEpoch i32 | magic i8 (=2) | crc u32 (CRC-32C of the bytes
//   from attributes to the end) | attributes i16 | lastOffsetDelta i32 | firstTimestamp i64 | maxTimestamp i64 |
//   producerId i64 | producerEpoch i16 | baseSequence i32 | count i32 | records…
// Record: length varint | attributes i8 | timestampDelta varlong | offsetDelta varint | keyLen varint | key |
//   valueLen varint | value | headerCount varint | headers…   (varints are zig-zag)
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <zlib.h>

#include "dxa_lz4.h"
#include "dxa_snappy.h"
#include "dxa_zstd.h"

namespace {

// largest decoded record-batch payload the host walker allocates (a batch's declared sizes are untrusted: a corrupt
// header must return an error code, never throw bad_alloc through the C entry points)
constexpr int64_t kMaxDecoded = (int64_t)1 << 31;

uint32_t g_crc_table[8][256];

// table for the portable path, built once (thread-safe static init)
bool crc_init() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    g_crc_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_crc_table[t][i] = (g_crc_table[t - 1][i] >> 8) ^ g_crc_table[0][g_crc_table[t - 1][i] & 0xff];
  return true;
}

uint32_t crc32c_sw(const uint8_t* p, size_t n, uint32_t c) {
  static const bool init = crc_init();
  (void)init;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= c;
    c = g_crc_table[7][w & 0xff] ^ g_crc_table[6][(w >> 8) & 0xff] ^ g_crc_table[5][(w >> 16) & 0xff] ^
        g_crc_table[4][(w >> 24) & 0xff] ^ g_crc_table[3][(w >> 32) & 0xff] ^ g_crc_table[2][(w >> 40) & 0xff] ^
        g_crc_table[1][(w >> 48) & 0xff] ^ g_crc_table[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ g_crc_table[0][(c ^ *p++) & 0xff];
  return c;
}

#if defined(__x86_64__)
// SSE4.2 crc32 computes exactly CRC-32C (Castagnoli): one 8-byte step per instruction, ~8 GB/s per core against
// ~2.5 GB/s for the slice-by-8 table path (Kafka's check.crcs covers every record batch a fetch returns)
__attribute__((target("sse4.2"))) uint32_t crc32c_hw(const uint8_t* p, size_t n, uint32_t c) {
  uint64_t c64 = c;
  while (n && ((uintptr_t)p & 7)) { c64 = __builtin_ia32_crc32qi((uint32_t)c64, *p++); --n; }
  while (n >= 32) {
    uint64_t w0, w1, w2, w3;
    std::memcpy(&w0, p, 8); std::memcpy(&w1, p + 8, 8); std::memcpy(&w2, p + 16, 8); std::memcpy(&w3, p + 24, 8);
    c64 = __builtin_ia32_crc32di(c64, w0);
    c64 = __builtin_ia32_crc32di(c64, w1);
    c64 = __builtin_ia32_crc32di(c64, w2);
    c64 = __builtin_ia32_crc32di(c64, w3);
    p += 32;
    n -= 32;
  }
  while (n >= 8) { uint64_t w; std::memcpy(&w, p, 8); c64 = __builtin_ia32_crc32di(c64, w); p += 8; n -= 8; }
  while (n--) c64 = __builtin_ia32_crc32qi((uint32_t)c64, *p++);
  return (uint32_t)c64;
}
const bool g_has_sse42 = __builtin_cpu_supports("sse4.2");
#endif

uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (g_has_sse42) return crc32c_hw(p, n, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
#endif
  return crc32c_sw(p, n, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

inline int64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return (int64_t)v;
}
inline int32_t be32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]); }
inline int16_t be16(const uint8_t* p) { return (int16_t)((uint16_t)p[0] << 8 | p[1]); }

inline bool varlong(const uint8_t*& p, const uint8_t* end, int64_t& out) {
  uint64_t v = 0;
  int shift = 0;
  while (p < end) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      out = (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
      return true;
    }
    shift += 7;
    if (shift > 63) return false;
  }
  return false;
}

void put_varlong(std::string& o, int64_t v) {
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  while (z >= 0x80) { o.push_back((char)((z & 0x7f) | 0x80)); z >>= 7; }
  o.push_back((char)z);
}
void put_be(std::string& o, uint64_t v, int bytes) {
  for (int i = bytes - 1; i >= 0; --i) o.push_back((char)((v >> (8 * i)) & 0xff));
}

bool gunzip(const uint8_t* src, size_t n, std::string& out) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, 15 + 32) != Z_OK) return false;
  zs.next_in = const_cast<uint8_t*>(src);
  zs.avail_in = (uInt)n;
  char buf[1 << 16];
  int rc;
  do {
    zs.next_out = (Bytef*)buf;
    zs.avail_out = sizeof buf;
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) { inflateEnd(&zs); return false; }
    out.append(buf, sizeof buf - zs.avail_out);
  } while (rc != Z_STREAM_END);
  inflateEnd(&zs);
  return true;
}

// Kafka codec 3: the records section is one LZ4 frame (Java producers omit the content size).
bool lz4_unframe(const uint8_t* src, size_t n, std::string& out) {
  int64_t content = -1, frame_end = 0;
  int32_t max_block = 0;
  const int64_t nb = dxa::lz4::frame_blocks(src, (int64_t)n, nullptr, nullptr, nullptr, 0, &content, &max_block,
                                            &frame_end);
  if (nb == -1) return false;
  const int64_t cap = content >= 0 ? content : (nb > 0 ? nb : 1) * (int64_t)max_block;
  if (cap > kMaxDecoded || (content >= 0 && content > (nb > 0 ? nb : 1) * (int64_t)max_block)) return false;
  out.resize((size_t)cap);
  const int64_t m = dxa::lz4::decompress_frame(src, (int64_t)n, (uint8_t*)&out[0], cap);
  if (m < 0) return false;
  out.resize((size_t)m);
  return true;
}

bool gzip_bytes(const std::string& in, std::string& out) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  out.resize(deflateBound(&zs, (uLong)in.size()) + 32);
  zs.next_in = (Bytef*)in.data();
  zs.avail_in = (uInt)in.size();
  zs.next_out = (Bytef*)&out[0];
  zs.avail_out = (uInt)out.size();
  const int rc = deflate(&zs, Z_FINISH);
  deflateEnd(&zs);
  if (rc != Z_STREAM_END) return false;
  out.resize(zs.total_out);
  return true;
}

struct Sink {
  // two-pass: count/size, then copy
  bool write;
  uint8_t* vals;
  int64_t* offs;       // [n+1] value start offsets in vals
  int64_t* rec_offs;   // Kafka offset of each record (may be null)
  int64_t n = 0;
  int64_t bytes = 0;
};

// returns 0 ok, <0 error; walks the records of one (decompressed) record area
int walk_records(const uint8_t* p, const uint8_t* end, int32_t count, int64_t base_offset, int64_t min_offset,
                 Sink& s) {
  for (int32_t r = 0; r < count; ++r) {
    int64_t len, tsd, od, klen, vlen, nh;
    if (!varlong(p, end, len)) return -10;
    const uint8_t* rec_end = p + len;
    if (rec_end > end) return -11;
    ++p;                               // attributes
    if (!varlong(p, rec_end, tsd) || !varlong(p, rec_end, od) || !varlong(p, rec_end, klen)) return -12;
    if (klen > 0) p += klen;
    if (!varlong(p, rec_end, vlen)) return -13;
    const uint8_t* v = p;
    if (vlen > 0) p += vlen;
    if (p > rec_end) return -14;
    (void)nh;
    const int64_t off = base_offset + od;
    if (off >= min_offset && vlen >= 0) {
      if (s.write) {
        s.offs[s.n] = s.bytes;
        std::memcpy(s.vals + s.bytes, v, (size_t)vlen);
        if (s.rec_offs) s.rec_offs[s.n] = off;
      }
      s.bytes += vlen;
      ++s.n;
    }
    p = rec_end;
  }
  return 0;
}

int walk_batches(const uint8_t* data, int64_t len, int64_t min_offset, int64_t max_records, Sink& s,
                 int64_t* next_offset, int verify_crc) {
  const uint8_t* p = data;
  const uint8_t* end = data + len;
  *next_offset = min_offset;
  while (end - p >= 61) {
    const int64_t base = be64(p);
    const int32_t blen = be32(p + 8);
    if (blen < 49 || end - (p + 12) < blen) break;     // a partial trailing batch is normal in Fetch responses
    const uint8_t* b = p + 12;                         // partitionLeaderEpoch
    const int8_t magic = (int8_t)b[4];
    if (magic != 2) return -2;
    const uint32_t crc = (uint32_t)be32(b + 5);
    const uint8_t* attrs_p = b + 9;
    const uint8_t* bend = p + 12 + blen;
    if (verify_crc && crc32c(attrs_p, (size_t)(bend - attrs_p)) != crc) return -3;
    const int16_t attrs = be16(attrs_p);
    const int32_t last_delta = be32(attrs_p + 2);
    const int32_t count = be32(attrs_p + 2 + 4 + 8 + 8 + 8 + 2 + 4);
    const uint8_t* recs = attrs_p + 2 + 4 + 8 + 8 + 8 + 2 + 4 + 4;
    const bool control = (attrs >> 5) & 1;
    if (!control && base + last_delta >= min_offset) {
      if (max_records >= 0 && s.n >= max_records) break;
      const int codec = attrs & 7;
      int rc;
      if (codec == 0) {
        rc = walk_records(recs, bend, count, base, min_offset, s);
      } else if (codec == 1) {
        std::string raw;
        if (!gunzip(recs, (size_t)(bend - recs), raw)) return -4;
        rc = walk_records((const uint8_t*)raw.data(), (const uint8_t*)raw.data() + raw.size(), count, base,
                          min_offset, s);
      } else if (codec == 3) {
        std::string raw;
        if (!lz4_unframe(recs, (size_t)(bend - recs), raw)) return -6;
        rc = walk_records((const uint8_t*)raw.data(), (const uint8_t*)raw.data() + raw.size(), count, base,
                          min_offset, s);
      } else if (codec == 2) {
        // snappy: snappy-java's xerial stream (Java producers) or one raw block (librdkafka)
        const int64_t m = dxa::snappy::payload_length(recs, bend - recs);
        if (m < 0 || m > kMaxDecoded) return -6;
        std::string raw((size_t)m, '\0');
        if (dxa::snappy::decompress_payload(recs, bend - recs, (uint8_t*)&raw[0], m) != m) return -6;
        rc = walk_records((const uint8_t*)raw.data(), (const uint8_t*)raw.data() + raw.size(), count, base,
                          min_offset, s);
      } else if (codec == 4) {
        // zstd: one frame (zstd-jni's ZstdOutputStream; no content size, so decode into a bound-sized buffer)
        const int64_t bound = dxa::zstd::decompressed_bound(recs, bend - recs);
        if (bound < 0 || bound > kMaxDecoded) return -6;
        std::string raw((size_t)bound, '\0');
        const int64_t m = dxa::zstd::decompress(recs, bend - recs, (uint8_t*)&raw[0], bound);
        if (m < 0) return -6;
        raw.resize((size_t)m);
        rc = walk_records((const uint8_t*)raw.data(), (const uint8_t*)raw.data() + raw.size(), count, base,
                          min_offset, s);
      } else {
        return -5;                                     // unknown codec
      }
      if (rc) return rc;
    }
    *next_offset = base + last_delta + 1 > *next_offset ? base + last_delta + 1 : *next_offset;
    p = bend;
  }
  return 0;
}

// ---- device-decode plan -----------------------------------------------------------------------------------------
// Walks only the record-batch headers and LZ4 frame block headers of a Fetch record set (no record bytes), so the
// records themselves are decompressed and framed on the GPU (lz4.hip + kafka_records.hip).  Each block gets an
// output slot: the frame's maximum block size for LZ4 blocks (every block of a frame but the last is full, so a
// frame's bytes are contiguous from its first slot), its own length for stored data, the gzip trailer's ISIZE for
// a gzip member (kind 2: inflated by inflate.hip).  Returns 0, or
// -2 bad magic, -3 CRC, -5 codec the GPU path does not take (snappy / zstd, odd gzip headers), -7 malformed LZ4 / snappy / zstd payload,
// -8 dependent-block frame, -9 offset deltas that are not 0..count-1 (compacted batch) — the caller decodes such
// fetches on the host.
struct Plan {
  bool write;
  int32_t* b_count; int64_t* b_base; int32_t* b_skip; int32_t* b_first; int32_t* b_nblk; int64_t* b_rec0;
  int64_t* k_comp_off; int32_t* k_comp_len; uint8_t* k_stored; int64_t* k_out_off; int64_t* k_cap;
  // per batch: the CRC-covered range (attributes .. end, offset from the set start) and the stored CRC-32C, for the
  // device-side check (kafka_crc_kernel); optional
  int64_t* b_crc_off = nullptr; int32_t* b_crc_len = nullptr; int32_t* b_crc = nullptr;
  int64_t nbat = 0, nblk = 0, nrec = 0, out_bytes = 0;
  int32_t max_block = 0;
};

// Length of a gzip member header (RFC 1952 2.3: ID1 ID2 CM FLG MTIME XFL OS, then FEXTRA / FNAME / FCOMMENT /
// FHCRC as flagged), or -1 when it is not a deflate gzip header.
int64_t gzip_header_len(const uint8_t* p, int64_t n) {
  if (n < 10 || p[0] != 0x1f || p[1] != 0x8b || p[2] != 8) return -1;
  const uint8_t flg = p[3];
  if (flg & 0xe0) return -1;                         // reserved bits
  int64_t k = 10;
  if (flg & 4) {                                     // FEXTRA
    if (k + 2 > n) return -1;
    k += 2 + ((int64_t)p[k] | ((int64_t)p[k + 1] << 8));
  }
  for (int f : {8, 16}) {                            // FNAME, FCOMMENT: zero-terminated
    if (flg & f) {
      while (k < n && p[k]) ++k;
      if (k >= n) return -1;
      ++k;
    }
  }
  if (flg & 2) k += 2;                               // FHCRC
  return k <= n ? k : -1;
}

int plan_batches(const uint8_t* data, int64_t len, int64_t min_offset, Plan& pl, int64_t* next_offset,
                 int verify_crc) {
  const uint8_t* p = data;
  const uint8_t* end = data + len;
  *next_offset = min_offset;
  while (end - p >= 61) {
    const int64_t base = be64(p);
    const int32_t blen = be32(p + 8);
    if (blen < 49 || end - (p + 12) < blen) break;
    const uint8_t* b = p + 12;
    if ((int8_t)b[4] != 2) return -2;
    const uint32_t crc = (uint32_t)be32(b + 5);
    const uint8_t* attrs_p = b + 9;
    const uint8_t* bend = p + 12 + blen;
    if (verify_crc && crc32c(attrs_p, (size_t)(bend - attrs_p)) != crc) return -3;
    const int16_t attrs = be16(attrs_p);
    const int32_t last_delta = be32(attrs_p + 2);
    const int32_t count = be32(attrs_p + 2 + 4 + 8 + 8 + 8 + 2 + 4);
    const uint8_t* recs = attrs_p + 2 + 4 + 8 + 8 + 8 + 2 + 4 + 4;
    const bool control = (attrs >> 5) & 1;
    if (!control && count > 0 && base + last_delta >= min_offset) {
      if (last_delta != count - 1) return -9;
      const int codec = attrs & 7;
      const int32_t skip = min_offset > base ? (int32_t)(min_offset - base) : 0;
      const int64_t first = pl.nblk;
      if (codec == 0) {
        if (pl.write) {
          pl.k_comp_off[pl.nblk] = recs - data;
          pl.k_comp_len[pl.nblk] = (int32_t)(bend - recs);
          pl.k_stored[pl.nblk] = 1;
          pl.k_out_off[pl.nblk] = pl.out_bytes;
          pl.k_cap[pl.nblk] = bend - recs;
        }
        pl.out_bytes += bend - recs;
        ++pl.nblk;
      } else if (codec == 3) {
        int64_t content = -1, fend = 0;
        int32_t mb = 0;
        const int64_t nb = dxa::lz4::frame_blocks(recs, bend - recs, nullptr, nullptr, nullptr, 0, &content, &mb,
                                                  &fend);
        if (nb == -2) return -8;
        if (nb < 0) return -7;
        if (pl.write) {
          dxa::lz4::frame_blocks(recs, bend - recs, pl.k_comp_off + pl.nblk, pl.k_comp_len + pl.nblk,
                                 pl.k_stored + pl.nblk, nb, &content, &mb, &fend);
          for (int64_t k = 0; k < nb; ++k) {
            pl.k_comp_off[pl.nblk + k] += recs - data;
            pl.k_out_off[pl.nblk + k] = pl.out_bytes + k * (int64_t)mb;
            pl.k_cap[pl.nblk + k] = mb;
          }
        }
        if (mb > pl.max_block) pl.max_block = mb;
        pl.out_bytes += nb * (int64_t)mb;
        pl.nblk += nb;
      } else if (codec == 1) {
        // gzip (Java GZIPOutputStream: one member): the device inflates the deflate data between the header and
        // the 8-byte trailer, whose ISIZE is the exact decompressed size (inflate.hip)
        const int64_t hdr = gzip_header_len(recs, bend - recs);
        if (hdr < 0 || bend - recs < hdr + 8) return -5;
        const uint8_t* t = bend - 4;
        const int64_t isize = (int64_t)t[0] | ((int64_t)t[1] << 8) | ((int64_t)t[2] << 16) | ((int64_t)t[3] << 24);
        if (isize > INT32_MAX) return -5;
        if (pl.write) {
          pl.k_comp_off[pl.nblk] = recs + hdr - data;
          pl.k_comp_len[pl.nblk] = (int32_t)(bend - 8 - (recs + hdr));
          pl.k_stored[pl.nblk] = 2;
          pl.k_out_off[pl.nblk] = pl.out_bytes;
          pl.k_cap[pl.nblk] = isize;
        }
        if (isize > pl.max_block) pl.max_block = (int32_t)isize;
        pl.out_bytes += isize;
        ++pl.nblk;
      } else if (codec == 2) {
        // snappy: every xerial chunk (or the one raw block) is an independent raw block with its exact size in
        // its varint preamble — kind 3, decoded by snappy.hip
        if (dxa::snappy::is_xerial(recs, bend - recs)) {
          const int64_t nc = dxa::snappy::xerial_chunks(recs, bend - recs, nullptr, nullptr, nullptr, 0);
          if (nc < 0) return -7;
          std::vector<int64_t> co((size_t)nc), ol((size_t)nc);
          std::vector<int32_t> cl((size_t)nc);
          dxa::snappy::xerial_chunks(recs, bend - recs, co.data(), cl.data(), ol.data(), nc);
          for (int64_t k = 0; k < nc; ++k) {
            if (pl.write) {
              pl.k_comp_off[pl.nblk] = recs + co[(size_t)k] - data;
              pl.k_comp_len[pl.nblk] = cl[(size_t)k];
              pl.k_stored[pl.nblk] = 3;
              pl.k_out_off[pl.nblk] = pl.out_bytes;
              pl.k_cap[pl.nblk] = ol[(size_t)k];
            }
            if (ol[(size_t)k] > pl.max_block) pl.max_block = (int32_t)ol[(size_t)k];
            pl.out_bytes += ol[(size_t)k];
            ++pl.nblk;
          }
        } else {
          const int64_t m = dxa::snappy::raw_length(recs, bend - recs, nullptr);
          if (m < 0) return -7;
          if (pl.write) {
            pl.k_comp_off[pl.nblk] = recs - data;
            pl.k_comp_len[pl.nblk] = (int32_t)(bend - recs);
            pl.k_stored[pl.nblk] = 3;
            pl.k_out_off[pl.nblk] = pl.out_bytes;
            pl.k_cap[pl.nblk] = m;
          }
          if (m > pl.max_block) pl.max_block = (int32_t)m;
          pl.out_bytes += m;
          ++pl.nblk;
        }
      } else if (codec == 4) {
        // zstd: one slot per frame (its blocks share the window, repeat offsets and entropy tables, so one wave
        // decodes the whole frame — zstd.hip); the slot is the frame's bound and the kernel reports the size
        const uint8_t* f = recs;
        while (f < bend) {
          dxa::zstd::FrameInfo fi;
          const int fr = dxa::zstd::frame_info(f, bend - f, &fi);
          if (fr == -2) return -5;                     // dictionary frames: host decoder only
          if (fr != 0) return -7;                      // malformed (incl. a content size beyond its blocks)
          if (fi.bound > INT32_MAX) return -7;         // a slot's capacity is an int32 (k_cap, max_block)
          if (pl.write) {
            pl.k_comp_off[pl.nblk] = f - data;
            pl.k_comp_len[pl.nblk] = (int32_t)fi.end;
            pl.k_stored[pl.nblk] = 4;
            pl.k_out_off[pl.nblk] = pl.out_bytes;
            pl.k_cap[pl.nblk] = fi.bound;
          }
          if (fi.bound > pl.max_block) pl.max_block = (int32_t)fi.bound;
          pl.out_bytes += fi.bound;
          ++pl.nblk;
          f += fi.end;
        }
      } else {
        return -5;
      }
      if (pl.write) {
        pl.b_count[pl.nbat] = count;
        pl.b_base[pl.nbat] = base;
        pl.b_skip[pl.nbat] = skip;
        pl.b_first[pl.nbat] = (int32_t)first;
        pl.b_nblk[pl.nbat] = (int32_t)(pl.nblk - first);
        pl.b_rec0[pl.nbat] = pl.nrec;
        if (pl.b_crc_off) {
          pl.b_crc_off[pl.nbat] = attrs_p - data;
          pl.b_crc_len[pl.nbat] = (int32_t)(bend - attrs_p);
          pl.b_crc[pl.nbat] = (int32_t)crc;
        }
      }
      pl.nrec += count - skip;
      ++pl.nbat;
    }
    *next_offset = base + last_delta + 1 > *next_offset ? base + last_delta + 1 : *next_offset;
    p = bend;
  }
  return 0;
}

template <typename F>
void parallel_sets(int64_t nsets, int threads, F f) {
  const int T = threads > 0 ? (int)std::min<int64_t>(threads, nsets) : 1;
  if (T <= 1) {
    for (int64_t k = 0; k < nsets; ++k) f(k);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < T; ++t)
    pool.emplace_back([&, t]() { for (int64_t k = t; k < nsets; k += T) f(k); });
  for (auto& th : pool) th.join();
}
}  // namespace

extern "C" {

// Device-decode plan of a Fetch record set: call with null arrays to size them (counts[0..3] = batches, blocks,
// records, output bytes; counts[4] = largest block capacity), then again to fill them.
__attribute__((visibility("default"))) int dxa_kafka_plan(const uint8_t* data, int64_t len, int64_t min_offset,
                                                         int verify_crc, int64_t* counts, int64_t* next_offset,
                                                         int32_t* b_count, int64_t* b_base, int32_t* b_skip,
                                                         int32_t* b_first, int32_t* b_nblk, int64_t* b_rec0,
                                                         int64_t* k_comp_off, int32_t* k_comp_len, uint8_t* k_stored,
                                                         int64_t* k_out_off, int64_t* k_cap, int64_t* b_crc_off,
                                                         int32_t* b_crc_len, int32_t* b_crc) {
  Plan pl{b_count != nullptr, b_count, b_base, b_skip, b_first, b_nblk, b_rec0,
          k_comp_off, k_comp_len, k_stored, k_out_off, k_cap, b_crc_off, b_crc_len, b_crc};
  const int rc = plan_batches(data, len, min_offset, pl, next_offset, verify_crc);
  counts[0] = pl.nbat;
  counts[1] = pl.nblk;
  counts[2] = pl.nrec;
  counts[3] = pl.out_bytes;
  counts[4] = pl.max_block;
  return rc;
}


__attribute__((visibility("default"))) uint32_t dxa_crc32c(const uint8_t* p, int64_t n) { return crc32c(p, (size_t)n); }

// Pass 1: how many records at offset >= min_offset and how many value bytes.
__attribute__((visibility("default"))) int dxa_kafka_count(const uint8_t* data, int64_t len, int64_t min_offset,
                                                          int64_t* n_records, int64_t* n_bytes, int64_t* next_offset,
                                                          int verify_crc) {
  Sink s{false, nullptr, nullptr, nullptr};
  const int rc = walk_batches(data, len, min_offset, -1, s, next_offset, verify_crc);
  *n_records = s.n;
  *n_bytes = s.bytes;
  return rc;
}

// Pass 2: copy values back to back into vals (caller adds padding), offs[n+1], rec_offs[n] (optional).
__attribute__((visibility("default"))) int dxa_kafka_extract(const uint8_t* data, int64_t len, int64_t min_offset,
                                                            uint8_t* vals, int64_t* offs, int64_t* rec_offs,
                                                            int64_t* next_offset) {
  Sink s{true, vals, offs, rec_offs};
  const int rc = walk_batches(data, len, min_offset, -1, s, next_offset, 0);
  offs[s.n] = s.bytes;
  return rc;
}

int64_t dxa_zstd_compress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t level, int32_t flags);
int64_t dxa_zstd_compress_bound(int64_t n);

// Encode n values (vals + offs[n+1]) as one v2 batch (codec 0 none, 1 gzip, 2 snappy, 3 lz4, 4 zstd) (baseOffset 0);
// returns malloc'd bytes.  lz4: one frame of `block_size` blocks at compression `level` (Kafka
// compression.lz4.level); zstd: one frame at zstd `level`.
__attribute__((visibility("default"))) uint8_t* dxa_kafka_encode_lz4(const uint8_t* vals, const int64_t* offs,
                                                                    int64_t n, int64_t timestamp_ms, int32_t codec,
                                                                    int32_t level, int32_t block_size,
                                                                    int64_t* out_len);

__attribute__((visibility("default"))) uint8_t* dxa_kafka_encode(const uint8_t* vals, const int64_t* offs, int64_t n,
                                                                int64_t timestamp_ms, int32_t codec,
                                                                int64_t* out_len) {
  return dxa_kafka_encode_lz4(vals, offs, n, timestamp_ms, codec, 1, 64 * 1024, out_len);
}

__attribute__((visibility("default"))) uint8_t* dxa_kafka_encode_lz4(const uint8_t* vals, const int64_t* offs,
                                                                    int64_t n, int64_t timestamp_ms, int32_t codec,
                                                                    int32_t level, int32_t block_size,
                                                                    int64_t* out_len) {
  std::string recs;
  for (int64_t i = 0; i < n; ++i) {
    std::string r;
    r.push_back(0);                     // attributes
    put_varlong(r, 0);                  // timestampDelta
    put_varlong(r, i);                  // offsetDelta
    put_varlong(r, -1);                 // null key
    const int64_t vlen = offs[i + 1] - offs[i];
    put_varlong(r, vlen);
    r.append((const char*)vals + offs[i], (size_t)vlen);
    put_varlong(r, 0);                  // no headers
    put_varlong(recs, (int64_t)r.size());
    recs += r;
  }
  if (codec == 1) {
    std::string z;
    if (!gzip_bytes(recs, z)) return nullptr;
    recs.swap(z);
  } else if (codec == 3) {
    std::string z((size_t)dxa::lz4::frame_bound((int64_t)recs.size(), block_size), '\0');
    const int64_t m = dxa::lz4::compress_frame((const uint8_t*)recs.data(), (int64_t)recs.size(), (uint8_t*)&z[0],
                                               (int64_t)z.size(), block_size, 1, level);
    if (m < 0) return nullptr;
    z.resize((size_t)m);
    recs.swap(z);
  } else if (codec == 2) {
    // snappy as the Java producer writes it: snappy-java's xerial stream of 32 KiB chunks
    std::string z((size_t)dxa::snappy::xerial_bound((int64_t)recs.size()), '\0');
    const int64_t m = dxa::snappy::xerial_compress((const uint8_t*)recs.data(), (int64_t)recs.size(),
                                                   (uint8_t*)&z[0]);
    z.resize((size_t)m);
    recs.swap(z);
  } else if (codec == 4) {
    // zstd at `level` (Kafka compression.zstd.level, default 3) through the system libzstd, as zstd-jni would
    const int64_t bound = dxa_zstd_compress_bound((int64_t)recs.size());
    if (bound < 0) return nullptr;
    std::string z((size_t)bound, '\0');
    const int64_t m = dxa_zstd_compress((const uint8_t*)recs.data(), (int64_t)recs.size(), (uint8_t*)&z[0], bound,
                                        level, 0);          // no content size, no checksum: zstd-jni's stream
    if (m < 0) return nullptr;
    z.resize((size_t)m);
    recs.swap(z);
  } else if (codec != 0) {
    return nullptr;
  }
  std::string body;                     // from attributes to the end (CRC domain)
  put_be(body, (uint64_t)codec, 2);     // attributes: compression codec, CreateTime
  put_be(body, (uint64_t)(n > 0 ? n - 1 : 0), 4);
  put_be(body, (uint64_t)timestamp_ms, 8);
  put_be(body, (uint64_t)timestamp_ms, 8);
  put_be(body, (uint64_t)-1, 8);        // producerId
  put_be(body, (uint64_t)-1, 2);        // producerEpoch
  put_be(body, (uint64_t)-1, 4);        // baseSequence
  put_be(body, (uint64_t)n, 4);
  body += recs;
  std::string out;
  put_be(out, 0, 8);                    // baseOffset (assigned by the broker)
  put_be(out, (uint64_t)(4 + 1 + 4 + body.size()), 4);
  put_be(out, 0, 4);                    // partitionLeaderEpoch
  out.push_back(2);                     // magic
  put_be(out, crc32c((const uint8_t*)body.data(), body.size()), 4);
  out += body;
  uint8_t* p = (uint8_t*)std::malloc(out.size());
  std::memcpy(p, out.data(), out.size());
  *out_len = (int64_t)out.size();
  return p;
}

// Plans of many record sets at once (one per partition fetch), each set on its own worker: the header walk is a
// chain of cache misses (one batch header every few KiB), so sets are walked in parallel.  count: per set
// [nbat, nblk, nrec, out_bytes] (set_counts[4*s..]) and next offsets; fill: the sets' plans back to back in the
// merged arrays (block / output / record indices rebased, block payload offsets relative to `data`).

__attribute__((visibility("default"))) int dxa_kafka_plan_count(const uint8_t* data, int64_t nsets,
                                                               const int64_t* set_off, const int64_t* set_len,
                                                               const int64_t* min_off, int verify_crc, int threads,
                                                               int64_t* set_counts, int64_t* next_off) {
  std::vector<int> rcs((size_t)nsets, 0);
  parallel_sets(nsets, threads, [&](int64_t k) {
    Plan pl{false, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
            nullptr};
    rcs[(size_t)k] = plan_batches(data + set_off[k], set_len[k], min_off[k], pl, &next_off[k], verify_crc);
    set_counts[4 * k] = pl.nbat;
    set_counts[4 * k + 1] = pl.nblk;
    set_counts[4 * k + 2] = pl.nrec;
    set_counts[4 * k + 3] = pl.out_bytes;
  });
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

__attribute__((visibility("default"))) int dxa_kafka_plan_fill(const uint8_t* data, int64_t nsets,
                                                              const int64_t* set_off, const int64_t* set_len,
                                                              const int64_t* min_off, int threads,
                                                              const int64_t* set_counts, int32_t* b_count,
                                                              int64_t* b_base, int32_t* b_skip, int32_t* b_first,
                                                              int32_t* b_nblk, int64_t* b_rec0, int64_t* k_comp_off,
                                                              int32_t* k_comp_len, uint8_t* k_stored,
                                                              int64_t* k_out_off, int64_t* k_cap, int64_t* b_crc_off,
                                                              int32_t* b_crc_len, int32_t* b_crc) {
  std::vector<int64_t> base((size_t)(4 * (nsets + 1)), 0);
  for (int64_t k = 0; k < nsets; ++k)
    for (int j = 0; j < 4; ++j) base[(size_t)(4 * (k + 1) + j)] = base[(size_t)(4 * k + j)] + set_counts[4 * k + j];
  std::vector<int> rcs((size_t)nsets, 0);
  parallel_sets(nsets, threads, [&](int64_t k) {
    const int64_t b0 = base[(size_t)(4 * k)], k0 = base[(size_t)(4 * k + 1)], r0 = base[(size_t)(4 * k + 2)],
                  o0 = base[(size_t)(4 * k + 3)];
    Plan pl{true, b_count + b0, b_base + b0, b_skip + b0, b_first + b0, b_nblk + b0, b_rec0 + b0,
            k_comp_off + k0, k_comp_len + k0, k_stored + k0, k_out_off + k0, k_cap + k0,
            b_crc_off ? b_crc_off + b0 : nullptr, b_crc_len ? b_crc_len + b0 : nullptr, b_crc ? b_crc + b0 : nullptr};
    int64_t nxt = 0;
    rcs[(size_t)k] = plan_batches(data + set_off[k], set_len[k], min_off[k], pl, &nxt, 0);
    for (int64_t i = 0; i < pl.nbat; ++i) {
      b_first[b0 + i] += (int32_t)k0;
      b_rec0[b0 + i] += r0;
      if (b_crc_off) b_crc_off[b0 + i] += set_off[k];
    }
    for (int64_t i = 0; i < pl.nblk; ++i) {
      k_comp_off[k0 + i] += set_off[k];
      k_out_off[k0 + i] += o0;
    }
  });
  for (int rc : rcs)
    if (rc) return rc;
  return 0;
}

// A producer's stream of record batches as a Fetch response returns them: n values cut into batches of
// `per_batch` records (the producer's batch.size), each one v2 batch (codec / level / LZ4 block size as above)
// with broker-assigned base offsets from `base_offset`; `threads` encode batches in parallel.  Returns malloc'd
// bytes (batches back to back).
__attribute__((visibility("default"))) uint8_t* dxa_kafka_encode_stream(const uint8_t* vals, const int64_t* offs,
                                                                       int64_t n, int64_t per_batch,
                                                                       int64_t base_offset, int64_t timestamp_ms,
                                                                       int32_t codec, int32_t level,
                                                                       int32_t block_size, int32_t threads,
                                                                       int64_t* out_len) {
  if (per_batch <= 0) return nullptr;
  const int64_t nbat = (n + per_batch - 1) / per_batch;
  std::vector<uint8_t*> parts((size_t)nbat, nullptr);
  std::vector<int64_t> lens((size_t)nbat, 0);
  const int T = threads > 0 ? threads : 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < T; ++t) {
    pool.emplace_back([&, t]() {
      for (int64_t b = t; b < nbat; b += T) {
        const int64_t lo = b * per_batch, hi = lo + per_batch < n ? lo + per_batch : n;
        parts[(size_t)b] = dxa_kafka_encode_lz4(vals, offs + lo, hi - lo, timestamp_ms, codec, level, block_size,
                                                &lens[(size_t)b]);
      }
    });
  }
  for (auto& th : pool) th.join();
  int64_t total = 0;
  bool ok = true;
  for (int64_t b = 0; b < nbat; ++b) {
    ok = ok && parts[(size_t)b] != nullptr;
    total += lens[(size_t)b];
  }
  uint8_t* out = ok ? (uint8_t*)std::malloc((size_t)(total > 0 ? total : 1)) : nullptr;
  int64_t pos = 0;
  for (int64_t b = 0; b < nbat; ++b) {
    if (out) {
      std::memcpy(out + pos, parts[(size_t)b], (size_t)lens[(size_t)b]);
      const int64_t base = base_offset + b * per_batch;
      for (int k = 0; k < 8; ++k) out[pos + k] = (uint8_t)((uint64_t)base >> (56 - 8 * k));
      pos += lens[(size_t)b];
    }
    std::free(parts[(size_t)b]);
  }
  *out_len = total;
  return out;
}
}
