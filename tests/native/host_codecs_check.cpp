// Native self-check of the host codecs, built with AddressSanitizer + UBSan by tests/test_native_sanitizers.py:
// Kafka record-batch encode → decode round trips for every codec (incl. truncated and corrupted input), CRC-32C
// vectors, LZ4 frame round trips plus decoding of random garbage / truncated frames, and the Java double formatter.  Exit code 0 = clean.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
uint32_t dxa_crc32c(const uint8_t* p, int64_t n);
int dxa_kafka_count(const uint8_t* data, int64_t len, int64_t min_offset, int64_t* n_records, int64_t* n_bytes,
                    int64_t* next_offset, int verify_crc);
int dxa_kafka_extract(const uint8_t* data, int64_t len, int64_t min_offset, uint8_t* vals, int64_t* offs,
                      int64_t* rec_offs, int64_t* next_offset);
uint8_t* dxa_kafka_encode(const uint8_t* vals, const int64_t* offs, int64_t n, int64_t timestamp_ms, int32_t codec,
                          int64_t* out_len);
int64_t dxa_lz4_frame_bound(int64_t n, int32_t block_size);
int64_t dxa_lz4_compress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t block_size,
                               int32_t threads);
int64_t dxa_lz4_decompress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t dxa_lz4_decompress_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
void dxa_host_free(void* p);
int dxa_java_double(double d, char* out, int cap);
}

static int failures = 0;
#define CHECK(c) do { if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } } while (0)

static void kafka_roundtrip(int nvals, uint32_t seed, int codec) {
  std::vector<std::string> vals;
  std::string all;
  std::vector<int64_t> offs{0};
  for (int i = 0; i < nvals; ++i) {
    seed = seed * 1664525u + 1013904223u;
    std::string v(seed % 300, (char)('a' + i % 26));
    vals.push_back(v);
    all += v;
    offs.push_back((int64_t)all.size());
  }
  int64_t blen = 0;
  uint8_t* batch = dxa_kafka_encode((const uint8_t*)all.data(), offs.data(), nvals, 1234, codec, &blen);
  for (int64_t cut = blen; cut >= 0; cut -= (blen / 7 + 1)) {       // whole batch, then truncated prefixes
    int64_t n = 0, nb = 0, nxt = 0;
    const int rc = dxa_kafka_count(batch, cut, 0, &n, &nb, &nxt, 1);
    CHECK(rc == 0);
    if (rc != 0) std::fprintf(stderr, "codec %d nvals %d cut %lld rc %d\n", codec, nvals, (long long)cut, rc);
    if (cut < blen) { CHECK(n == 0); continue; }
    CHECK(n == nvals && nb == (int64_t)all.size());
    std::vector<uint8_t> out((size_t)nb + 16);
    std::vector<int64_t> o((size_t)n + 1), ro((size_t)(n > 0 ? n : 1));
    CHECK(dxa_kafka_extract(batch, cut, 0, out.data(), o.data(), ro.data(), &nxt) == 0);
    for (int i = 0; i < nvals; ++i) {
      CHECK(std::string((const char*)out.data() + o[i], (size_t)(o[i + 1] - o[i])) == vals[i]);
      CHECK(ro[i] == i);
    }
  }
  if (blen > 70) {                                                    // corrupted payload → CRC error, no crash
    std::vector<uint8_t> bad(batch, batch + blen);
    bad[blen - 1] ^= 0x5a;
    int64_t n = 0, nb = 0, nxt = 0;
    CHECK(dxa_kafka_count(bad.data(), blen, 0, &n, &nb, &nxt, 1) == -3);
  }
  dxa_host_free(batch);
}

static void lz4_checks(uint32_t seed) {
  for (int64_t n : {0, 1, 12, 13, 100, 5000, 70000}) {
    std::vector<uint8_t> src((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      seed = seed * 1664525u + 1013904223u;
      src[(size_t)i] = (uint8_t)((seed >> 24) % (i % 3 == 0 ? 4 : 200));
    }
    for (int32_t bs : {1024, 65536}) {
      std::vector<uint8_t> f((size_t)dxa_lz4_frame_bound(n, bs));
      const int64_t m = dxa_lz4_compress_frame(src.data(), n, f.data(), (int64_t)f.size(), bs, 2);
      CHECK(m > 0);
      std::vector<uint8_t> out((size_t)n + 1);
      CHECK(dxa_lz4_decompress_frame(f.data(), m, out.data(), n) == n);
      CHECK(n == 0 || std::memcmp(out.data(), src.data(), (size_t)n) == 0);
      for (int64_t cut = 1; cut < m; cut += m / 5 + 1) {            // truncated frames fail cleanly
        CHECK(dxa_lz4_decompress_frame(f.data(), cut, out.data(), n) < 0);
      }
    }
  }
  std::vector<uint8_t> junk(4096), out(8192);                        // garbage blocks: errors, never overruns
  for (int t = 0; t < 200; ++t) {
    for (auto& b : junk) { seed = seed * 1664525u + 1013904223u; b = (uint8_t)(seed >> 24); }
    const int64_t r = dxa_lz4_decompress_block(junk.data(), (int64_t)(seed % 4096), out.data(), (int64_t)out.size());
    CHECK(r >= -1 && r <= (int64_t)out.size());
  }
}

extern "C" {
int64_t dxa_snappy_compress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t xerial);
int64_t dxa_snappy_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t dxa_zstd_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t dxa_zstd_compress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t level, int32_t flags);
}

// snappy and zstd: round trips, truncated streams and garbage inputs return errors, never overrun
static void snappy_zstd_checks(uint32_t seed) {
  for (int64_t n : {0, 1, 100, 5000, 40000, 140000}) {
    std::vector<uint8_t> src((size_t)n);
    for (auto& b : src) { seed = seed * 1664525u + 1013904223u; b = (uint8_t)"{\"a\":12,"[(seed >> 24) % 8]; }
    for (int xer : {0, 1}) {
      std::vector<uint8_t> z((size_t)(256 + 2 * n)), out((size_t)n + 1);
      const int64_t m = dxa_snappy_compress(src.data(), n, z.data(), (int64_t)z.size(), xer);
      CHECK(m > 0);
      CHECK(dxa_snappy_decompress(z.data(), m, out.data(), n) == n);
      CHECK(n == 0 || std::memcmp(out.data(), src.data(), (size_t)n) == 0);
      for (int64_t cut = 0; cut < m; cut += 1 + m / 7) CHECK(dxa_snappy_decompress(z.data(), cut, out.data(), n) != n ||
                                                              cut == m);
    }
    std::vector<uint8_t> z((size_t)(1024 + 2 * n)), out((size_t)n + 64);
    const int64_t m = dxa_zstd_compress(src.data(), n, z.data(), (int64_t)z.size(), 3, 0);
    if (m > 0) {                                                 // libzstd present
      CHECK(dxa_zstd_decompress(z.data(), m, out.data(), (int64_t)out.size()) == n);
      CHECK(n == 0 || std::memcmp(out.data(), src.data(), (size_t)n) == 0);
      for (int64_t cut = 0; cut < m; cut += 1 + m / 9) {
        const int64_t r = dxa_zstd_decompress(z.data(), cut, out.data(), (int64_t)out.size());
        CHECK(r < 0 || r <= (int64_t)out.size());
      }
    }
  }
  std::vector<uint8_t> junk(4096), out(70000);
  for (int t = 0; t < 300; ++t) {
    for (auto& b : junk) { seed = seed * 1664525u + 1013904223u; b = (uint8_t)(seed >> 24); }
    if (t & 1) { junk[0] = 0x28; junk[1] = 0xB5; junk[2] = 0x2F; junk[3] = 0xFD; }   // zstd magic, garbage body
    const int64_t len = (int64_t)(seed % 4096);
    const int64_t r = dxa_zstd_decompress(junk.data(), len, out.data(), (int64_t)out.size());
    CHECK(r <= (int64_t)out.size());
    const int64_t q = dxa_snappy_decompress(junk.data(), len, out.data(), (int64_t)out.size());
    CHECK(q <= (int64_t)out.size());
  }
}

// A CRC-valid v2 batch around a records payload whose declared decoded size is absurd: a zstd frame header claiming
// 2^62 bytes of content, a snappy varint claiming 2^31-1 bytes for 4 literal bytes.  The walker must return an error
// code (no bad_alloc / length_error escaping the C entry point, no huge allocation).
static void put_be(std::vector<uint8_t>& b, uint64_t v, int n) {
  for (int k = n - 1; k >= 0; --k) b.push_back((uint8_t)(v >> (8 * k)));
}
static std::vector<uint8_t> raw_batch(const std::vector<uint8_t>& payload, int codec) {
  std::vector<uint8_t> tail;
  put_be(tail, (uint64_t)codec, 2);        // attributes
  put_be(tail, 0, 4);                      // last offset delta (one record)
  put_be(tail, 1234, 8);
  put_be(tail, 1234, 8);
  put_be(tail, ~0ull, 8);                  // producer id -1
  put_be(tail, 0xffff, 2);
  put_be(tail, 0xffffffffu, 4);
  put_be(tail, 1, 4);                      // record count
  tail.insert(tail.end(), payload.begin(), payload.end());
  std::vector<uint8_t> b;
  put_be(b, 0, 8);
  put_be(b, (uint64_t)(4 + 1 + 4 + tail.size()), 4);
  put_be(b, 0, 4);                         // partition leader epoch
  b.push_back(2);                          // magic
  put_be(b, dxa_crc32c(tail.data(), (int64_t)tail.size()), 4);
  b.insert(b.end(), tail.begin(), tail.end());
  return b;
}
static void oversized_declared_sizes() {
  // zstd: single-segment frame, 8-byte content size 2^62, one raw block "abcd"
  std::vector<uint8_t> z = {0x28, 0xB5, 0x2F, 0xFD, 0xE0};
  for (int k = 0; k < 8; ++k) z.push_back((uint8_t)(((uint64_t)1 << 62) >> (8 * k)));
  const uint32_t bh = 1 | (0 << 1) | (4 << 3);
  z.push_back((uint8_t)bh); z.push_back((uint8_t)(bh >> 8)); z.push_back((uint8_t)(bh >> 16));
  for (char c : std::string("abcd")) z.push_back((uint8_t)c);
  std::vector<uint8_t> out(64);
  CHECK(dxa_zstd_decompress(z.data(), (int64_t)z.size(), out.data(), (int64_t)out.size()) < 0);
  // snappy: varint 2^31-1, then a 4-byte literal
  std::vector<uint8_t> s = {0xFF, 0xFF, 0xFF, 0xFF, 0x07, 3 << 2, 'a', 'b', 'c', 'd'};
  CHECK(dxa_snappy_decompress(s.data(), (int64_t)s.size(), out.data(), (int64_t)out.size()) < 0);
  for (const auto& pc : {std::make_pair(z, 4), std::make_pair(s, 2)}) {
    const std::vector<uint8_t> b = raw_batch(pc.first, pc.second);
    int64_t n = 0, nb = 0, nxt = 0;
    const int rc = dxa_kafka_count(b.data(), (int64_t)b.size(), 0, &n, &nb, &nxt, 1);
    CHECK(rc == -6);
    if (rc != -6) std::fprintf(stderr, "oversized codec %d rc %d\n", pc.second, rc);
  }
}

int main() {
  snappy_zstd_checks(5u);
  oversized_declared_sizes();
  CHECK(dxa_crc32c((const uint8_t*)"123456789", 9) == 0xE3069283u);
  CHECK(dxa_crc32c((const uint8_t*)"", 0) == 0u);
  for (int codec : {0, 1, 2, 3, 4})
    for (int n : {0, 1, 2, 17, 200}) kafka_roundtrip(n, 7u + n, codec);
  lz4_checks(99u);
  char buf[64];
  // (subnormal extremes such as Double.MIN_VALUE are not checked: Java pads to two digits there — "4.9E-324" —
  // while the shortest-digit formatter prints "5.0E-324")
  const double vals[] = {0.0, -0.0, 1.0, 0.1, 1e7, 1e-3, 123.456, 2.2250738585072014e-308, 1.7976931348623157e308,
                         NAN, INFINITY};
  const char* want[] = {"0.0", "-0.0", "1.0", "0.1", "1.0E7", "0.001", "123.456", "2.2250738585072014E-308",
                        "1.7976931348623157E308", "\"NaN\"", "\"Infinity\""};
  for (int i = 0; i < 11; ++i) {
    const int k = dxa_java_double(vals[i], buf, 64);
    CHECK(std::string(buf, (size_t)k) == want[i]);
  }
  std::printf("host codecs: %d failures\n", failures);
  return failures ? 1 : 0;
}
