// Schema-directed JSON → columnar parser for gfx950 (kernel K3 in SURVEY.md §2.F).
//
// Replaces the reference's per-row `from_json(Raw, rawSchema)` (DataProcessing/datax-host/src/main/scala/datax/
// processor/CommonProcessorFactory.scala:93).  One lane owns one record: records are 100–800 B, a batch holds
// 10^5–10^7 of them, so a 256-lane block per 256 records gives thousands of workgroups (≫ 256 CUs × 8 XCDs).
// Each lane streams its record through a 64-byte window in LDS (see Reader) and runs a branch-light state
// machine; keys are first matched against the key the schema order predicts (8-byte compares), otherwise
// FNV-hashed and resolved against a small open-addressed (parent-node, key-hash) lookup table.
//
// Output is written straight into column slots: 8-byte values (int64 / double bits / timestamp µs), string VIEWS
// (start offset into the same device buffer + length — the parser never copies string bytes; strings containing
// escapes are un-escaped in place, which only ever shrinks them), and a validity byte per (node,row).
//
// Semantics: missing field / JSON null / type mismatch → null for that field; a syntactically malformed record
// → every field of the row null and row_ok=0 (the reference is "tolerant to mismatched input schema").
#include "dxa_common.h"
#include <type_traits>
#include "decimal_dd.h"
#include "dxa_ts.h"

namespace {

enum : int32_t {
  FT_STRUCT = 0, FT_BOOL = 1, FT_LONG = 2, FT_DOUBLE = 3, FT_STRING = 4, FT_RAW = 5,
  FT_TIMESTAMP = 6, FT_INT = 7, FT_DATE = 8, FT_DECIMAL = 9,   // FT_DECIMAL: the number token's text (decimal.hip)
  FT_SKIP = 10,               // a pruned field: matched in schema order (cheap), its value skipped unstored
};

struct ParseArgs {
  uint8_t* buf;                 // raw bytes (16-B padded at the end)
  const int64_t* offs;          // [n+1] record boundaries
  int64_t n;
  const uint64_t* lut_keys;     // [lut_cap] 0 = empty
  const int32_t* lut_node;      // [lut_cap]
  int32_t lut_cap;
  const int32_t* node_type;     // [nnodes]
  const int32_t* val_slot;      // [nnodes] → value row (-1: none)
  const int32_t* len_slot;      // [nnodes] → length row (-1: none)
  int32_t nnodes;
  int64_t* vals;                // [nval][n]
  int32_t* lens;                // [nlen][n]
  uint8_t* valid;               // [nnodes][n]  (pre-zeroed)
  uint8_t* row_ok;              // [n]
  // key-order speculation: producers emit keys in a fixed order, so the next key is predicted (schema order,
  // re-synchronised after every key) and checked with 8-byte compares instead of a byte-serial hash
  const int32_t* first_child;   // [nnodes] first kept child of a struct node (-1: none)
  const int32_t* next_sib;      // [nnodes] next kept sibling (-1: none)
  const int32_t* key_word;      // [nnodes] offset (in u64 words) of the node's key text
  const int32_t* key_len;       // [nnodes] key length in bytes
  const uint64_t* key_words;    // key texts, zero padded to 8-byte words
  int32_t nkey_words;
  const int64_t* ends;          // [n] record ends when records are not back to back (Kafka values), else null;
                                // offs[n] is then the end of the bytes
  // outputs split in two: rows of the assembled columns (value slots < nkv, length slots < nkl, nodes < nkn) in
  // vals / lens / valid, the parsed-but-dropped ones (column pruning) in vals2 / lens2 / valid2, so a retained
  // column pins only its own batch's kept rows
  int64_t* vals2;
  int32_t* lens2;
  uint8_t* valid2;
  int32_t nkv, nkl, nkn;
  // (value slot, length slot) of every assembled string-like field: zeroed per row first, so a missing or null
  // string is an empty view at offset 0, never a stale address (the buffers are not pre-filled)
  const int32_t* zslots;
  int32_t nz;
};

// The same arguments as explicitly global (address space 1) pointers.  Pointers read out of a by-value struct
// argument are otherwise generic, and every record-byte load and column store becomes a FLAT op — counted in
// both vmcnt and lgkmcnt, so each LDS wait also drains the lane's outstanding global loads.
#define G1 __attribute__((address_space(1)))
typedef G1 uint8_t gu8;
struct GArgs {
  gu8* buf;
  const G1 int64_t* offs;
  int64_t n;
  const G1 uint64_t* lut_keys;
  const G1 int32_t* lut_node;
  int32_t lut_cap;
  const G1 int32_t* node_type;
  const G1 int32_t* val_slot;
  const G1 int32_t* len_slot;
  int32_t nnodes;
  G1 int64_t* vals;
  G1 int32_t* lens;
  gu8* valid;
  gu8* row_ok;
  const G1 int32_t* first_child;
  const G1 int32_t* next_sib;
  const G1 int32_t* key_word;
  const G1 int32_t* key_len;
  const G1 uint64_t* key_words;
  int32_t nkey_words;
  const G1 int64_t* ends;
  G1 int64_t* vals2;
  G1 int32_t* lens2;
  gu8* valid2;
  int32_t nkv, nkl, nkn;
  const G1 int32_t* zslots;
  int32_t nz;
  // row pointers of value slot v, length slot l, node k
  __device__ __forceinline__ G1 int64_t* vrow(int v) const {
    return v < nkv ? vals + (int64_t)v * n : vals2 + (int64_t)(v - nkv) * n;
  }
  __device__ __forceinline__ G1 int32_t* lrow(int l) const {
    return l < nkl ? lens + (int64_t)l * n : lens2 + (int64_t)(l - nkl) * n;
  }
  __device__ __forceinline__ gu8* drow(int k) const {
    return k < nkn ? valid + (int64_t)k * n : valid2 + (int64_t)(k - nkn) * n;
  }
};

__device__ __forceinline__ GArgs to_global(const ParseArgs& p) {
  GArgs g;
  g.buf = (gu8*)p.buf;
  g.offs = (const G1 int64_t*)p.offs;
  g.n = p.n;
  g.lut_keys = (const G1 uint64_t*)p.lut_keys;
  g.lut_node = (const G1 int32_t*)p.lut_node;
  g.lut_cap = p.lut_cap;
  g.node_type = (const G1 int32_t*)p.node_type;
  g.val_slot = (const G1 int32_t*)p.val_slot;
  g.len_slot = (const G1 int32_t*)p.len_slot;
  g.nnodes = p.nnodes;
  g.vals = (G1 int64_t*)p.vals;
  g.lens = (G1 int32_t*)p.lens;
  g.valid = (gu8*)p.valid;
  g.row_ok = (gu8*)p.row_ok;
  g.first_child = (const G1 int32_t*)p.first_child;
  g.next_sib = (const G1 int32_t*)p.next_sib;
  g.key_word = (const G1 int32_t*)p.key_word;
  g.key_len = (const G1 int32_t*)p.key_len;
  g.key_words = (const G1 uint64_t*)p.key_words;
  g.nkey_words = p.nkey_words;
  g.ends = (const G1 int64_t*)p.ends;
  g.vals2 = (G1 int64_t*)p.vals2;
  g.lens2 = (G1 int32_t*)p.lens2;
  g.valid2 = (gu8*)p.valid2;
  g.nkv = p.nkv;
  g.nkl = p.nkl;
  g.nkn = p.nkn;
  g.zslots = (const G1 int32_t*)p.zslots;
  g.nz = p.nz;
  return g;
}

__constant__ uint64_t kPow10i[9] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                    100000000ull};
__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};


// Schema tables (node info, key texts, key lookup table) as seen by the parse loop.  With LDS=true the workgroup
// first copies them into LDS: every field does ~9 table reads, and as VMEM loads they go through the same per-CU
// address path the record bytes saturate; from LDS they are broadcast reads.
#define G3 __attribute__((address_space(3)))
template <bool LDS>
struct Tables {
  typedef typename std::conditional<LDS, const G3 int32_t*, const G1 int32_t*>::type I32P;
  typedef typename std::conditional<LDS, const G3 uint64_t*, const G1 uint64_t*>::type U64P;
  I32P node_type, val_slot, len_slot, first_child, next_sib, key_word, key_len, lut_node;
  U64P key_words, lut_keys;
  int32_t lut_cap;
};

__host__ __device__ inline int64_t tables_lds_bytes(int32_t nnodes, int32_t nkw, int32_t lut_cap) {
  return (int64_t)nkw * 8 + (int64_t)lut_cap * 8 + (int64_t)(8 * nnodes + lut_cap) * 4;
}

template <bool LDS>
__device__ __forceinline__ Tables<LDS> load_tables(const GArgs& a);

template <>
__device__ __forceinline__ Tables<false> load_tables<false>(const GArgs& a) {
  Tables<false> t;
  t.node_type = a.node_type; t.val_slot = a.val_slot; t.len_slot = a.len_slot;
  t.first_child = a.first_child; t.next_sib = a.next_sib; t.key_word = a.key_word; t.key_len = a.key_len;
  t.lut_node = a.lut_node; t.key_words = a.key_words; t.lut_keys = a.lut_keys; t.lut_cap = a.lut_cap;
  return t;
}

extern __shared__ uint64_t dyn_lds[];

template <>
__device__ __forceinline__ Tables<true> load_tables<true>(const GArgs& a) {
  G3 uint64_t* u64 = (G3 uint64_t*)dyn_lds;
  G3 uint64_t* kw = u64;
  G3 uint64_t* lk = u64 + a.nkey_words;
  G3 int32_t* i32 = (G3 int32_t*)(lk + a.lut_cap);
  const int nn = a.nnodes;
  G3 int32_t* arr[7] = {i32, i32 + nn, i32 + 2 * nn, i32 + 3 * nn, i32 + 4 * nn, i32 + 5 * nn, i32 + 6 * nn};
  G3 int32_t* ln = i32 + 8 * nn;
  for (int i = threadIdx.x; i < a.nkey_words; i += blockDim.x) kw[i] = a.key_words[i];
  for (int i = threadIdx.x; i < a.lut_cap; i += blockDim.x) { lk[i] = a.lut_keys[i]; ln[i] = a.lut_node[i]; }
  for (int i = threadIdx.x; i < nn; i += blockDim.x) {
    arr[0][i] = a.node_type[i]; arr[1][i] = a.val_slot[i]; arr[2][i] = a.len_slot[i];
    arr[3][i] = a.first_child[i]; arr[4][i] = a.next_sib[i]; arr[5][i] = a.key_word[i]; arr[6][i] = a.key_len[i];
  }
  __syncthreads();
  Tables<true> t;
  t.node_type = arr[0]; t.val_slot = arr[1]; t.len_slot = arr[2]; t.first_child = arr[3]; t.next_sib = arr[4];
  t.key_word = arr[5]; t.key_len = arr[6]; t.lut_node = ln; t.key_words = kw; t.lut_keys = lk;
  t.lut_cap = a.lut_cap;
  return t;
}

constexpr int kMaxDepth = 8;

// Per-lane byte window over the lane's record: 64 bytes in LDS ([dword][lane], conflict-free), topped up at the
// start of every field for all lanes that are low on bytes (``top_up``).  Lanes read 64 unrelated records, so each
// window load touches 64 cache lines and the per-CU address path, not VALU, bounds the parser.  Lanes sit at
// different offsets of their records, so per-lane refills stall a wave once per distinct refill point; refilling
// every low lane in the same instruction makes that about one stall per field.  (A 64-byte *register* window needs
// 217 VGPRs.)  Measured on the bench batch against the previous 32-byte register window (two global_load_dwordx4
// per refill): 2.30 -> 1.75 ms, VMEM reads per wave 344 -> 220, VALU per wave 24.3 K -> 14.7 K.
constexpr uint32_t kWin = 64;
#define G3U32 __attribute__((address_space(3))) uint32_t
struct Reader {
  gu8* buf;
  int64_t p, end;
  int64_t wb;                                             // window base offset (16-B aligned in memory)
  int64_t lim;                                            // window loads stay below buf + lim (last record + pad)
  G3U32* win;                                             // dword j of this lane's window at win[j * 256]

  __device__ __forceinline__ void fill(int64_t q) {
    const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(buf + q) & 15);
    wb = q - o;
    // near the end of the batch buffer, slide the window back so its loads stay inside the 16-B padding
    const int64_t hi = lim - (int64_t)kWin - (int64_t)(reinterpret_cast<uintptr_t>(buf + lim) & 15);
    if (wb > hi && hi >= 0) wb = hi;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const G1 u32x4* w = (const G1 u32x4*)(buf + wb);
    const u32x4 a = w[0], b = w[1], c = w[2], d = w[3];
    win[0 * 256] = a.x; win[1 * 256] = a.y; win[2 * 256] = a.z; win[3 * 256] = a.w;
    win[4 * 256] = b.x; win[5 * 256] = b.y; win[6 * 256] = b.z; win[7 * 256] = b.w;
    win[8 * 256] = c.x; win[9 * 256] = c.y; win[10 * 256] = c.z; win[11 * 256] = c.w;
    win[12 * 256] = d.x; win[13 * 256] = d.y; win[14 * 256] = d.z; win[15 * 256] = d.w;
  }
  // wave-synchronous refill: every lane with fewer than `need` bytes left in its window reloads in one instruction
  __device__ __forceinline__ void top_up(uint32_t need) {
    if ((uint64_t)(p - wb) > (uint64_t)(kWin - need)) fill(p);
  }
  __device__ __forceinline__ uint32_t at(int64_t q) {
    if ((uint64_t)(q - wb) >= kWin) fill(q);
    const uint32_t o = (uint32_t)(q - wb);
    return (win[(o >> 2) * 256] >> ((o & 3u) * 8u)) & 0xffu;
  }
  // 8 bytes starting at q (the batch buffer carries >= 16 bytes of tail padding); row 16 of the window is padding
  __device__ __forceinline__ uint64_t load8(int64_t q) {
    if ((uint64_t)(q - wb) > kWin - 8u) fill(q);
    const uint32_t o = (uint32_t)(q - wb);
    const uint32_t j = o >> 2, sh = o & 3u;
    const uint32_t d0 = win[j * 256], d1 = win[(j + 1) * 256], d2 = win[(j + 2) * 256];
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    return (uint64_t)lo | ((uint64_t)hi << 32);
  }
  __device__ __forceinline__ uint32_t cur() { return p < end ? at(p) : 0u; }
  // skip whitespace and return the character there (0 at the end): one window read in the common no-space case
  __device__ __forceinline__ uint32_t ws_cur() {
    while (p < end) {
      const uint32_t c = at(p);
      if (c != ' ' && c != '\n' && c != '\r' && c != '\t') return c;
      ++p;
    }
    return 0u;
  }
  __device__ __forceinline__ void skip_ws() {
    while (p < end) {
      const uint32_t c = at(p);
      if (c == ' ' || c == '\n' || c == '\r' || c == '\t') ++p; else break;
    }
  }
};

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }

// Does the key text at q equal the L-byte literal (followed by the closing quote)?
template <typename KW>
__device__ __forceinline__ bool key_matches(Reader& r, int64_t q, int64_t end, KW kw, int L) {
  if (q + L >= end) return false;
  int i = 0;
  for (; i + 8 <= L; i += 8)
    if (r.load8(q + i) != kw[i >> 3]) return false;
  const uint64_t tail = r.load8(q + i);
  const int rem = L - i;                                   // 0..7 bytes of key, then the quote
  const uint64_t mask = rem == 7 ? ~0ull : ((1ull << (8 * (rem + 1))) - 1);
  const uint64_t want = (rem ? kw[i >> 3] : 0ull) | ((uint64_t)'"' << (8 * rem));
  return ((tail ^ want) & mask) == 0;
}

// The expected key at q, its closing quote and — in the same 8-byte compare when it lies in the key's last word —
// the ':' right after it (compact JSON: no blank between key and colon).  Returns 0: no match; 1: key, quote and
// colon (r.p is then past the colon, and `next` holds the byte after the colon when that byte was in the compared
// word, else 256); 2: key and quote only (the colon, after blanks, is left to the generic path).
template <typename KW>
__device__ __forceinline__ int key_colon_matches(Reader& r, int64_t q, int64_t end, KW kw, int L, uint32_t& next) {
  if (q + L >= end) return 0;
  int i = 0;
  for (; i + 8 <= L; i += 8)
    if (r.load8(q + i) != kw[i >> 3]) return 0;
  const uint64_t tail = r.load8(q + i);
  const int rem = L - i;                                   // 0..7 key bytes, then the quote (and the colon)
  const uint64_t want = (rem ? kw[i >> 3] : 0ull) | ((uint64_t)'"' << (8 * rem));
  const uint64_t mq = rem == 7 ? ~0ull : ((1ull << (8 * (rem + 1))) - 1);
  if ((tail ^ want) & mq) return 0;
  next = 256u;
  if (rem == 7) {                                          // the colon is the next word's first byte
    if (q + L + 1 >= end || r.at(q + L + 1) != ':') return 2;
  } else {
    if (q + L + 1 >= end || ((tail >> (8 * (rem + 1))) & 0xffu) != ':') return 2;
    if (rem <= 5 && q + L + 2 < end) next = (uint32_t)((tail >> (8 * (rem + 2))) & 0xffu);
  }
  r.p = q + L + 2;
  return 1;
}

// After a member separator: the expected key's whole `"key":` at q (no blank before the quote or the colon), the
// pattern's words shifted out of the key words on the fly.  True: r.p is past the colon and `next` holds the byte
// after it when the last compared word holds it (256 otherwise).  False: nothing consumed.
template <typename KW>
__device__ __forceinline__ bool quote_key_colon(Reader& r, int64_t q, int64_t end, KW kw, int L, uint32_t& next) {
  const int P = L + 3;                                     // '"' key '"' ':'
  if (q + P > end) return false;
  const int nkw = (L + 7) >> 3;
  uint64_t x = 0;
  int j = 0;
  for (; 8 * j < P; ++j) {
    x = r.load8(q + 8 * j);
    uint64_t w = (j < nkw ? kw[j] << 8 : 0ull) | (j == 0 ? (uint64_t)'"' : (kw[j - 1] >> 56));
    const int t0 = L + 1 - 8 * j, t1 = L + 2 - 8 * j;     // the closing quote and the colon in this word
    if (t0 >= 0 && t0 < 8) w |= (uint64_t)'"' << (8 * t0);
    if (t1 >= 0 && t1 < 8) w |= (uint64_t)':' << (8 * t1);
    const int nb = P - 8 * j;                              // pattern bytes in this word
    const uint64_t m = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
    if ((x ^ w) & m) return false;
  }
  const int used = P - 8 * (j - 1);                        // pattern bytes in the last word (1..8)
  next = (used < 8 && q + P < end) ? (uint32_t)((x >> (8 * used)) & 0xffu) : 256u;
  r.p = q + P;
  return true;
}

// SWAR byte tests on 8 bytes (little-endian: byte 0 = first char): high bit of each byte lane flags the property.
__device__ __forceinline__ uint64_t swar_eq(uint64_t x, uint64_t pat) {
  const uint64_t v = x ^ pat;
  return (v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull;   // exact for the lowest flagged byte
}
__device__ __forceinline__ uint64_t swar_nondigit(uint64_t x) {
  return ((x + 0x4646464646464646ull) | (x - 0x3030303030303030ull)) & 0x8080808080808080ull;
}
// Value of the k (1..8) leading digit characters of x (byte 0 = most significant digit): the digits are shifted to
// the top bytes and the zero bytes below them read as leading '0's of an 8-digit number.
__device__ __forceinline__ uint64_t swar_digits(uint64_t x, int k) {
  uint64_t v = (x - 0x3030303030303030ull) << (8 * (8 - k));
  v = ((v & 0x0F0F0F0F0F0F0F0Full) * 2561) >> 8;
  v = ((v & 0x00FF00FF00FF00FFull) * 6553601) >> 16;
  return ((v & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
}

// Bytes below 0x20 (unescaped control characters); exact for the lowest flagged byte, like swar_eq.
__device__ __forceinline__ uint64_t swar_ctl(uint64_t x) {
  return (x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull;
}

// Scan a string whose opening quote is at r.p.  On return r.p is past the closing quote.  Eight bytes per step:
// the first quote, backslash or control character is found with SWAR compares (a string of ~10 chars is one or
// two steps).  An unescaped control character makes the record malformed (strict JSON, as Jackson's default).
// `after`: the byte following the closing quote when the compared word holds it (256 otherwise) — the caller's
// next token without another window read.
__device__ __forceinline__ bool scan_string(Reader& r, int64_t& s, int64_t& e, bool& esc, uint32_t& after) {
  ++r.p;
  s = r.p;
  esc = false;
  after = 256u;
  while (r.p < r.end) {
    const uint64_t x = r.load8(r.p);
    const uint64_t m = swar_eq(x, 0x2222222222222222ull) | swar_eq(x, 0x5C5C5C5C5C5C5C5Cull) | swar_ctl(x);
    if (m == 0) { r.p += 8; continue; }
    const int j = __builtin_ctzll(m) >> 3;
    r.p += j;
    if (r.p >= r.end) break;
    const uint32_t c = (uint32_t)((x >> (8 * j)) & 0xff);
    if (c == '"') {
      e = r.p;
      ++r.p;
      if (j < 7 && r.p < r.end) after = (uint32_t)((x >> (8 * (j + 1))) & 0xff);
      return true;
    }
    if (c < 0x20u) break;                                 // raw control character inside a string
    esc = true;
    if (r.p + 1 >= r.end) break;
    const uint32_t n = r.at(r.p + 1);                     // the escaped character must be one JSON defines
    if (n == 'u') {
      if (r.p + 6 > r.end) break;
      bool hex = true;
      for (int k = 2; k < 6; ++k) {
        const uint32_t h = r.at(r.p + k);
        hex &= (h - '0' < 10u) || ((h | 0x20u) - 'a' < 6u);
      }
      if (!hex) break;
      r.p += 6;
      continue;
    }
    if (!(n == '"' || n == '\\' || n == '/' || n == 'b' || n == 'f' || n == 'n' || n == 'r' || n == 't')) break;
    r.p += 2;                                             // backslash + escaped char
  }
  r.p = r.end;
  return false;
}
__device__ __forceinline__ bool scan_string(Reader& r, int64_t& s, int64_t& e, bool& esc) {
  uint32_t after;
  return scan_string(r, s, e, esc, after);
}

__device__ __forceinline__ uint32_t hexval(uint32_t c) {
  if (c - '0' < 10u) return c - '0';
  c |= 0x20u;
  if (c - 'a' < 6u) return c - 'a' + 10;
  return 0;
}

// Un-escape [s,e) in place; returns the decoded length.
__device__ __forceinline__ int64_t unescape_inplace(Reader& r, int64_t s, int64_t e) {
  gu8* b = r.buf;
  int64_t o = s;
  int64_t i = s;
  while (i < e) {
    uint32_t c = b[i];
    if (c != '\\') { b[o++] = (uint8_t)c; ++i; continue; }
    if (i + 1 >= e) break;
    const uint32_t n = b[i + 1];
    i += 2;
    switch (n) {
      case 'n': b[o++] = '\n'; break;
      case 't': b[o++] = '\t'; break;
      case 'r': b[o++] = '\r'; break;
      case 'b': b[o++] = '\b'; break;
      case 'f': b[o++] = '\f'; break;
      case 'u': {
        if (i + 4 > e) { i = e; break; }
        uint32_t cp = (hexval(b[i]) << 12) | (hexval(b[i + 1]) << 8) | (hexval(b[i + 2]) << 4) | hexval(b[i + 3]);
        i += 4;
        if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= e && b[i] == '\\' && b[i + 1] == 'u') {
          const uint32_t lo = (hexval(b[i + 2]) << 12) | (hexval(b[i + 3]) << 8) | (hexval(b[i + 4]) << 4) |
                              hexval(b[i + 5]);
          if (lo >= 0xDC00 && lo < 0xE000) {
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            i += 6;
          }
        }
        if (cp < 0x80) {
          b[o++] = (uint8_t)cp;
        } else if (cp < 0x800) {
          b[o++] = (uint8_t)(0xC0 | (cp >> 6));
          b[o++] = (uint8_t)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
          b[o++] = (uint8_t)(0xE0 | (cp >> 12));
          b[o++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
          b[o++] = (uint8_t)(0x80 | (cp & 0x3F));
        } else {
          b[o++] = (uint8_t)(0xF0 | (cp >> 18));
          b[o++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
          b[o++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
          b[o++] = (uint8_t)(0x80 | (cp & 0x3F));
        }
        break;
      }
      default: b[o++] = (uint8_t)n; break;  // \" \\ \/ and unknown
    }
  }
  r.wb = -256;  // window may cover rewritten bytes
  return o - s;
}

// Run of decimal digits at r.p, accumulated into (mant, nd, exp10) exactly as a digit-serial loop would: at most
// 19 significant digits kept (leading zeros are not significant); integer-part digits beyond that raise exp10 and
// set `lost`; fraction digits beyond it are dropped.  Eight characters per step (SWAR digit test + conversion).
// `first`: the run's first character; `term`: the character that ended it when the last compared word holds it
// (256 otherwise: the record's end, or a word boundary).
__device__ __forceinline__ bool scan_digits(Reader& r, uint64_t& mant, int& nd, int& exp10, bool& lost, bool frac,
                                            uint64_t& tail, int& nt, uint32_t& first, uint32_t& term) {
  bool any = false;
  term = 256u;
  while (r.p < r.end) {
    const uint64_t x = r.load8(r.p);
    const uint64_t nm = swar_nondigit(x);
    int k = nm ? (__builtin_ctzll(nm) >> 3) : 8;
    const bool clamped = k > r.end - r.p;
    if (clamped) k = (int)(r.end - r.p);
    if (!clamped && k < 8) term = (uint32_t)((x >> (8 * k)) & 0xff);
    if (k == 0) break;
    if (!any) first = (uint32_t)(x & 0xff);
    any = true;
    const uint64_t chunk = swar_digits(x, k);
    int sig = k;                                          // significant digits this chunk adds
    if (mant == 0) {
      if (chunk == 0) {
        sig = 0;
      } else {
        const uint64_t nz = (x - 0x3030303030303030ull) & ((k == 8) ? ~0ull : ((1ull << (8 * k)) - 1));
        sig = k - (__builtin_ctzll(nz) >> 3);           // drop leading zero digits
      }
    }
    if (nd + sig <= 19) {
      mant = mant * kPow10i[k] + chunk;
      nd += sig;
      if (frac) exp10 -= k;
      r.p += k;
    } else {
      // the 19-digit boundary falls inside this chunk: finish digit by digit
      for (int i = 0; i < k; ++i) {
        const uint32_t c = (uint32_t)((x >> (8 * i)) & 0xff);
        if (nd < 19) {
          mant = mant * 10 + (c - '0');
          if (mant) ++nd;
          if (frac) --exp10;
        } else {
          if (!frac) { ++exp10; lost = true; }
          if (nt < 19) { tail = tail * 10 + (c - '0'); ++nt; }   // the next 19 digits, for the rounding
        }
      }
      r.p += k;
    }
    if (k < 8) break;
  }
  return any;
}

// Parse a JSON number at r.p, whose first character c the caller has read.  Returns false on syntax error.
// `term`: the character after the number when a digit scan saw it (256: unknown).
__device__ __forceinline__ bool scan_number(Reader& r, uint32_t c, bool& is_int, bool& overflow, int64_t& iv,
                                            double& dv, uint32_t& term) {
  bool neg = false;
  if (c == '-') { neg = true; ++r.p; }
  uint64_t mant = 0, tail = 0;
  int nd = 0, exp10 = 0, nt = 0;
  bool lost = false;
  is_int = true;
  const int64_t s0 = r.p;
  uint32_t first = 0;
  if (!scan_digits(r, mant, nd, exp10, lost, false, tail, nt, first, term)) return false;
  if (first == '0' && r.p - s0 > 1) return false;                                     // JSON: no leading zeros
  if (term == 256u) term = r.cur();
  if (term == '.') {
    is_int = false;
    ++r.p;
    uint32_t f2;
    if (!scan_digits(r, mant, nd, exp10, lost, true, tail, nt, f2, term)) return false;
    if (term == 256u) term = r.cur();
  }
  if ((term | 0x20u) == 'e') {
    term = 256u;
    is_int = false;
    ++r.p;
    bool eneg = false;
    if (r.cur() == '-' || r.cur() == '+') { eneg = r.cur() == '-'; ++r.p; }
    int e = 0;
    bool ed = false;
    while (r.p < r.end && is_digit(r.at(r.p))) {
      ed = true;
      if (e < 100000) e = e * 10 + (int)(r.at(r.p) - '0');
      ++r.p;
    }
    if (!ed) return false;
    exp10 += eneg ? -e : e;
  }
  overflow = false;
  if (is_int) {
    if (lost) overflow = true;
    else if (!neg && mant > 9223372036854775807ull) overflow = true;
    else if (neg && mant > 9223372036854775808ull) overflow = true;
    iv = neg ? (int64_t)(0ull - mant) : (int64_t)mant;
  }
  double d = (double)mant;
  if (exp10 != 0 || mant >= (1ull << 53) || tail != 0) {
    if (tail == 0 && mant < (1ull << 53) && exp10 > 0 && exp10 <= 22) d = d * kPow10[exp10];   // exact operands
    else if (tail == 0 && mant < (1ull << 53) && exp10 < 0 && exp10 >= -22) d = d / kPow10[-exp10];
    else if (mant == 0) d = 0.0;
    else if (exp10 > DXA_POW10_DD_MAX) d = __builtin_inf();
    else if (exp10 < DXA_POW10_DD_MIN) d = 0.0;
    else d = dxa_decimal_to_double(mant, exp10, tail, nt);
  }
  dv = neg ? -d : d;
  return true;
}

// true / false / null spelled out exactly (r.p at the first letter); advances past it.
__device__ __forceinline__ bool take_literal(Reader& r, uint32_t c) {
  const uint64_t x = r.load8(r.p);
  int L;
  bool good;
  if (c == 't') { L = 4; good = (x & 0xffffffffull) == 0x65757274ull; }             // "true"
  else if (c == 'n') { L = 4; good = (x & 0xffffffffull) == 0x6c6c756eull; }        // "null"
  else { L = 5; good = (x & 0xffffffffffull) == 0x65736c6166ull; }                   // "false"
  r.p += L;
  return good && r.p <= r.end;
}

// A run of digits at r.p, eight characters per step (SWAR digit test); false when there is none.  `first` / `term`
// as in scan_digits: the run's first character, and the character that ended it when a compared word held it (256
// otherwise).
__device__ __forceinline__ bool skip_digits(Reader& r, uint32_t& first, uint32_t& term) {
  const int64_t s = r.p;
  term = 256u;
  while (r.p < r.end) {
    const uint64_t x = r.load8(r.p);
    if (r.p == s) first = (uint32_t)(x & 0xff);
    const uint64_t nm = swar_nondigit(x);
    if (nm) {
      const int k = __builtin_ctzll(nm) >> 3;
      r.p += k;
      if (r.p < r.end) term = (uint32_t)((x >> (8 * k)) & 0xff);
      break;
    }
    r.p += 8;
  }
  if (r.p > r.end) { r.p = r.end; term = 256u; }          // digits past the record's end are not its own
  return r.p > s;
}
__device__ __forceinline__ bool skip_digits(Reader& r) {
  uint32_t first, term;
  return skip_digits(r, first, term);
}

// skip_number with the first character known (the caller's) and the following one reported when a digit scan saw
// it (`term`, 256 otherwise): a pruned number costs its digit words and no single-byte reads.
__device__ __forceinline__ bool skip_number(Reader& r, uint32_t c, uint32_t& term) {
  if (c == '-') ++r.p;
  const int64_t s = r.p;
  uint32_t first = 0;
  if (!skip_digits(r, first, term)) return false;
  if (first == '0' && r.p - s > 1) return false;           // leading zero
  if (term == 256u) term = r.cur();
  if (term == '.') {
    ++r.p;
    if (!skip_digits(r, first, term)) return false;
    if (term == 256u) term = r.cur();
  }
  if ((term | 0x20u) == 'e') {
    ++r.p;
    term = r.cur();
    if (term == '-' || term == '+') ++r.p;
    if (!skip_digits(r, first, term)) return false;
  }
  return true;
}

// A JSON number's syntax (-? int frac? exp?) without its value: the skipping paths (pruned fields, unknown keys)
// need no mantissa registers, and digit runs go eight at a time.
__device__ __forceinline__ bool skip_number(Reader& r) {
  if (r.cur() == '-') ++r.p;
  const int64_t s = r.p;
  if (!skip_digits(r)) return false;
  if (r.p - s > 1 && r.at(s) == '0') return false;        // leading zero
  uint32_t c = r.cur();
  if (c == '.') {
    ++r.p;
    if (!skip_digits(r)) return false;
    c = r.cur();
  }
  if ((c | 0x20u) == 'e') {
    ++r.p;
    c = r.cur();
    if (c == '-' || c == '+') ++r.p;
    if (!skip_digits(r)) return false;
  }
  return true;
}

// Skip any JSON value at r.p (strings, numbers, literals, nested containers), validating it as strictly as the
// fields that are parsed: an unknown subtree that is not well-formed JSON makes the record malformed, as it does for
// a tokenizing parser.  Containers are walked with an explicit state machine; the container kinds of up to 32
// nesting levels live in one bit mask (deeper input is rejected).
__device__ __forceinline__ bool skip_value(Reader& r) {
  uint32_t c = r.cur();
  if (c == '"') { int64_t s, e; bool esc; return scan_string(r, s, e, esc); }
  if (c == '-' || is_digit(c)) return skip_number(r);
  if (c == 't' || c == 'n' || c == 'f') return take_literal(r, c);
  if (c != '{' && c != '[') return false;
  enum { kVal, kValOrClose, kKey, kKeyOrClose, kColon, kSep };
  uint32_t obj = 0;                                       // bit d: level d is an object
  int depth = 0, st = kVal;
  while (true) {
    c = r.ws_cur();
    if (c == 0u) return false;
    switch (st) {
      case kVal:
      case kValOrClose:
        if (c == ']' && st == kValOrClose) goto close;
        if (c == '{' || c == '[') {
          if (depth == 32) return false;
          obj = (obj & ~(1u << depth)) | ((uint32_t)(c == '{') << depth);
          ++depth;
          ++r.p;
          st = c == '{' ? kKeyOrClose : kValOrClose;
          continue;
        }
        if (c == '"') { int64_t s, e; bool esc; if (!scan_string(r, s, e, esc)) return false; }
        else if (c == '-' || is_digit(c)) { if (!skip_number(r)) return false; }
        else if (c == 't' || c == 'n' || c == 'f') { if (!take_literal(r, c)) return false; }
        else return false;
        st = kSep;
        continue;
      case kKey:
      case kKeyOrClose:
        if (c == '}' && st == kKeyOrClose) goto close;
        if (c != '"') return false;
        { int64_t s, e; bool esc; if (!scan_string(r, s, e, esc)) return false; }
        st = kColon;
        continue;
      case kColon:
        if (c != ':') return false;
        ++r.p;
        st = kVal;
        continue;
      default:                                            // kSep: ',' or the current container's close
        if (c == ',') { ++r.p; st = (obj >> (depth - 1)) & 1 ? kKey : kVal; continue; }
        if (c == ((obj >> (depth - 1)) & 1 ? '}' : ']')) goto close;
        return false;
    }
  close:
    ++r.p;
    if (--depth == 0) return true;
    st = kSep;
  }
}

// Hash one escape sequence of a key (r.p at the backslash) as the bytes it decodes to, so "a\u0062" finds "ab".
__device__ __forceinline__ uint64_t hash_escape(Reader& r, uint64_t h) {
  ++r.p;
  if (r.p >= r.end) return h;
  const uint32_t n = r.at(r.p);
  ++r.p;
  uint32_t cp;
  switch (n) {
    case 'n': return dxa::fnv1a_step(h, '\n');
    case 't': return dxa::fnv1a_step(h, '\t');
    case 'r': return dxa::fnv1a_step(h, '\r');
    case 'b': return dxa::fnv1a_step(h, '\b');
    case 'f': return dxa::fnv1a_step(h, '\f');
    case 'u':
      if (r.p + 4 > r.end) { r.p = r.end; return h; }
      cp = (hexval(r.at(r.p)) << 12) | (hexval(r.at(r.p + 1)) << 8) | (hexval(r.at(r.p + 2)) << 4) |
           hexval(r.at(r.p + 3));
      r.p += 4;
      if (cp >= 0xD800 && cp < 0xDC00 && r.p + 6 <= r.end && r.at(r.p) == '\\' && r.at(r.p + 1) == 'u') {
        const uint32_t lo = (hexval(r.at(r.p + 2)) << 12) | (hexval(r.at(r.p + 3)) << 8) |
                            (hexval(r.at(r.p + 4)) << 4) | hexval(r.at(r.p + 5));
        if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); r.p += 6; }
      }
      if (cp < 0x80) return dxa::fnv1a_step(h, cp);
      if (cp < 0x800) {
        h = dxa::fnv1a_step(h, 0xC0 | (cp >> 6));
        return dxa::fnv1a_step(h, 0x80 | (cp & 0x3F));
      }
      if (cp < 0x10000) {
        h = dxa::fnv1a_step(h, 0xE0 | (cp >> 12));
        h = dxa::fnv1a_step(h, 0x80 | ((cp >> 6) & 0x3F));
        return dxa::fnv1a_step(h, 0x80 | (cp & 0x3F));
      }
      h = dxa::fnv1a_step(h, 0xF0 | (cp >> 18));
      h = dxa::fnv1a_step(h, 0x80 | ((cp >> 12) & 0x3F));
      h = dxa::fnv1a_step(h, 0x80 | ((cp >> 6) & 0x3F));
      return dxa::fnv1a_step(h, 0x80 | (cp & 0x3F));
    default: return dxa::fnv1a_step(h, n);            // \" \\ \/ and unknown escapes: the character itself
  }
}

template <typename T>
__device__ __forceinline__ int lookup(const T& a, int parent, uint64_t name_hash) {
  uint64_t k = dxa::fmix64(name_hash ^ ((uint64_t)(parent + 1) * dxa::kGold));
  if (k == 0) k = 1;
  const uint32_t mask = (uint32_t)a.lut_cap - 1u;
  uint32_t s = (uint32_t)k & mask;
  for (int probe = 0; probe < a.lut_cap; ++probe) {
    const uint64_t kk = a.lut_keys[s];
    if (kk == k) return a.lut_node[s];
    if (kk == 0) return -1;
    s = (s + 1) & mask;
  }
  return -1;
}

// Parse ISO-8601-ish text [s,e): YYYY-MM-DD[(T| )HH:MM[:SS[.ffffff]]][Z|(+|-)HH[:]MM]  → µs since epoch UTC.
__device__ __forceinline__ bool parse_iso_ts(Reader& rd, int64_t s, int64_t e, int64_t& out, bool date_only_ok) {
  struct B {
    Reader& r;
    __device__ __forceinline__ uint32_t operator[](int64_t i) const { return r.at(i); }
  } b{rd};
  auto num = [&](int64_t& i, int digits, int& v) -> bool {
    v = 0;
    for (int k = 0; k < digits; ++k) {
      if (i >= e || !is_digit(b[i])) return false;
      v = v * 10 + (b[i] - '0');
      ++i;
    }
    return true;
  };
  int64_t i = s;
  int y, mo, d, hh = 0, mi = 0, ss = 0;
  if (!num(i, 4, y) || i >= e || b[i] != '-') return false;
  ++i;
  if (!num(i, 2, mo) || i >= e || b[i] != '-') return false;
  ++i;
  if (!num(i, 2, d)) return false;
  int64_t frac_us = 0;
  int64_t tz_us = 0;
  if (i < e && (b[i] == 'T' || b[i] == ' ')) {
    ++i;
    if (!num(i, 2, hh) || i >= e || b[i] != ':') return false;
    ++i;
    if (!num(i, 2, mi)) return false;
    if (i < e && b[i] == ':') { ++i; if (!num(i, 2, ss)) return false; }
    if (i < e && b[i] == '.') {
      ++i;
      int64_t scale = 100000;
      while (i < e && is_digit(b[i])) { frac_us += (b[i] - '0') * scale; scale /= 10; ++i; }
    }
    if (i < e && b[i] == 'Z') ++i;
    else if (i < e && (b[i] == '+' || b[i] == '-')) {
      const bool neg = b[i] == '-';
      ++i;
      int th, tm = 0;
      if (!num(i, 2, th)) return false;
      if (i < e && b[i] == ':') ++i;
      if (i < e) { if (!num(i, 2, tm)) return false; }
      tz_us = ((int64_t)th * 3600 + tm * 60) * 1000000ll;
      if (neg) tz_us = -tz_us;
    }
  } else if (!date_only_ok) {
    return false;
  }
  if (i != e) return false;
  if (mo < 1 || mo > 12 || d < 1 || d > 31 || hh > 23 || mi > 59 || ss > 60) return false;
  const int64_t days = dxa::days_from_civil(y, (unsigned)mo, (unsigned)d);
  out = ((days * 86400 + hh * 3600 + mi * 60 + ss) * 1000000ll) + frac_us - tz_us;
  return true;
}

// Occupancy: with the LDS window the kernel needs ~103 VGPRs; amdgpu_waves_per_eu(5) caps it at 96 (2 dwords
// spilled on cold paths) for 5 waves per SIMD (LDS: 25 KiB per 256-lane workgroup).  Bench batch (2 M events,
// profiles/parse/parse_variants.md): register window 2.29 ms; LDS window 4 waves 1.76 ms; 5 waves 1.59 ms; 6 waves
// 1.76 ms (12 dwords spilled); top-up threshold 48/40/32/24/16/1 bytes -> 1.72/1.64/1.58/1.58/1.66/1.73 ms.
constexpr uint32_t kTopUp = 32;
typedef int16_t StackT;                               // node ids < 32767 (checked by the host entry point)
template <bool LDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void json_parse_kernel(ParseArgs pa) {
  const GArgs a = to_global(pa);
  const Tables<LDS> tb = load_tables<LDS>(a);                   // (LDS: whole workgroup, before any early exit)
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.n) return;
  for (int j = 0; j < a.nz; ++j) {
    a.vrow(a.zslots[2 * j])[row] = 0;
    a.lrow(a.zslots[2 * j + 1])[row] = 0;
  }
  const int64_t n = a.n;
  Reader r;
  r.buf = a.buf;
  r.p = a.offs[row];
  r.end = a.ends ? a.ends[row] : a.offs[row + 1];
  r.wb = -256;
  r.lim = a.offs[n] + 16;
  __shared__ uint32_t s_win[17][256];
  r.win = (G3U32*)&s_win[0][threadIdx.x];

  // schema-tracked nesting is kept in registers (deeper objects are skipped as unknown values)
  // nesting state in LDS, [level][lane] (consecutive lanes → consecutive banks): dynamically indexed per-lane
  // arrays would otherwise take 16 VGPRs (or a compiler-chosen LDS layout with bank conflicts)
  __shared__ StackT s_stack[kMaxDepth][256];
  __shared__ StackT s_expect[kMaxDepth][256];
  StackT* stack_ = &s_stack[0][threadIdx.x];
  StackT* expect_ = &s_expect[0][threadIdx.x];
#define stack(i) stack_[(i) * 256]
#define expect(i) expect_[(i) * 256]
  int depth = 0;
  bool ok = false;
  bool comma = false;         // the last token was a member separator
  int store_node = -1;        // skip_any: raw-JSON text of the skipped value goes to this node
  __shared__ uint64_t s_seen[256];                        // schema nodes (< 64) already assigned in this record
  s_seen[threadIdx.x] = 0;                                // (per lane in LDS: keeps the loop's VGPR budget)

  if (r.ws_cur() != '{') goto done;
  ++r.p;
  stack(0) = 0;  // root node
  expect(0) = tb.first_child[0];
  depth = 1;
  a.drow(0)[row] = 1;  // root struct present
  uint32_t nextc;             // the character after a scanned value when its scanner saw it (256: read it)
  while (true) {
    r.top_up(kTopUp);                        // key + typical value of the next field, all low lanes at once
    nextc = 256u;
    uint32_t c;
    int node;
    if (comma) {                             // the member after a separator: `"key":` of the expected key at once
      const int ex = expect(depth - 1);
      uint32_t nx = 256u;
      if (ex >= 0 && quote_key_colon(r, r.p, r.end, tb.key_words + tb.key_word[ex], tb.key_len[ex], nx)) {
        comma = false;
        store_node = -1;
        node = ex;
        expect(depth - 1) = tb.next_sib[node];
        c = (nx == 256u || nx == ' ' || nx == '\n' || nx == '\r' || nx == '\t') ? r.ws_cur() : nx;
        goto have_value;
      }
    }
    c = r.ws_cur();
    if (c == '}') {
      if (comma) break;       // trailing comma: {"a":1,}
      ++r.p;
      if (--depth == 0) { ok = true; break; }
      goto after_value;
    }
    if (c != '"') break;
    comma = false;
    store_node = -1;
    {
      // ---- key: speculate the expected key first, fall back to hashing the key text
     {
      ++r.p;
      node = -1;
      const int ex = expect(depth - 1);
      int km = 0;
      uint32_t nx = 256u;
      if (ex >= 0) km = key_colon_matches(r, r.p, r.end, tb.key_words + tb.key_word[ex], tb.key_len[ex], nx);
      if (km == 1) {                                      // `"key":` in one go: straight to the value
        node = ex;
        expect(depth - 1) = tb.next_sib[node];
        c = (nx == 256u || nx == ' ' || nx == '\n' || nx == '\r' || nx == '\t') ? r.ws_cur() : nx;
        goto have_value;
      }
      if (km == 2) {
        node = ex;
        r.p += tb.key_len[ex] + 1;
      } else {
        uint64_t h = dxa::kFnvBasis;
        bool closed = false;
        while (r.p < r.end) {
          const uint32_t kc = r.at(r.p);
          if (kc == '"') { ++r.p; closed = true; break; }
          if (kc == '\\') { h = hash_escape(r, h); continue; }
          h = dxa::fnv1a_step(h, kc);
          ++r.p;
        }
        if (!closed) break;
        node = lookup(tb, stack(depth - 1), h);
      }
      if (node >= 0) expect(depth - 1) = tb.next_sib[node];
      if (r.ws_cur() != ':') break;
      ++r.p;
      c = r.ws_cur();
     }
    have_value:
      if (node < 0) goto skip_any;
      const int t = tb.node_type[node] & 0xff;
      if (t == FT_SKIP) {
        // a pruned struct keeps its schema children (all FT_SKIP) in the plan: walk it like a struct, so key
        // speculation keeps matching inside it, and store nothing; other pruned values go to the skipper
        if (c == '{' && tb.first_child[node] >= 0 && depth < kMaxDepth) {
          expect(depth) = tb.first_child[node];
          stack(depth) = node;
          ++depth;
          ++r.p;
          continue;
        }
        goto skip_any;
      }
      const bool raw_arr = (tb.node_type[node] & 0x100) != 0;
      const int vs = tb.val_slot[node];
      const int ls = tb.len_slot[node];
      if (node < 64) {                                    // a repeated key: its last occurrence decides (null on a
        const uint64_t bit = 1ull << node;                // mismatch), as a tokenizing parser's last write would
        const uint64_t seen = s_seen[threadIdx.x];
        if (seen & bit) {
          a.drow(node)[row] = 0;
          const int sh = tb.node_type[node] >> 16;        // its timestamp shadow follows the last occurrence too
          if (sh) a.drow(sh)[row] = 0;
        }
        s_seen[threadIdx.x] = seen | bit;
      }
      if (c == '{' && t == FT_STRUCT) {
        if (depth >= kMaxDepth) goto skip_any;
        a.drow(node)[row] = 1;
        expect(depth) = tb.first_child[node];
        stack(depth) = node;
        ++depth;
        ++r.p;
        continue;
      }
      if (c == '{' || c == '[') {
        if ((t == FT_STRING || (t == FT_RAW && (c == '[') == raw_arr)) && ls >= 0) store_node = node;
        goto skip_any;
      }
      if (c == '"') {
        int64_t s, e;
        bool esc;
        if (!scan_string(r, s, e, esc, nextc)) break;
        if (t == FT_STRING) {
          const int64_t len = esc ? unescape_inplace(r, s, e) : (e - s);
          a.vrow(vs)[row] = s;
          a.lrow(ls)[row] = (int32_t)len;
          a.drow(node)[row] = 1;
          const int sh = tb.node_type[node] >> 16;      // timestamp shadow: stringToTimestamp of this field, here
          if (sh) {                                       // while its bytes are in cache (no separate kernel)
            int64_t us;
            if (dxa::string_to_ts((const uint8_t*)(r.buf + s), (int32_t)len, us)) {
              a.vrow(tb.val_slot[sh])[row] = us;
              a.drow(sh)[row] = 1;
            }
          }
        } else if (t == FT_TIMESTAMP || t == FT_DATE) {
          int64_t us;
          if (parse_iso_ts(r, s, e, us, true)) {
            a.vrow(vs)[row] = (t == FT_DATE) ? (us >= 0 ? us / 86400000000ll
                                                                     : -((-us + 86399999999ll) / 86400000000ll))
                                                           : us;
            a.drow(node)[row] = 1;
          }
        }
        goto after_value;
      }
      if (c == '-' || is_digit(c)) {
        const int64_t s = r.p;
        bool is_int, of;
        int64_t iv = 0;
        double dv = 0.0;
        if (!scan_number(r, c, is_int, of, iv, dv, nextc)) break;
        if (t == FT_LONG || t == FT_INT) {
          if (is_int && !of && (t == FT_LONG || (iv >= -2147483648ll && iv <= 2147483647ll))) {
            a.vrow(vs)[row] = iv;
            a.drow(node)[row] = 1;
          }
        } else if (t == FT_DOUBLE) {
          a.vrow(vs)[row] = __double_as_longlong(dv);
          a.drow(node)[row] = 1;
        } else if (t == FT_TIMESTAMP) {
          if (is_int && !of) {
            a.vrow(vs)[row] = iv * 1000000ll;
            a.drow(node)[row] = 1;
          }
        } else if (t == FT_STRING || t == FT_DECIMAL) {
          a.vrow(vs)[row] = s;
          a.lrow(ls)[row] = (int32_t)(r.p - s);
          a.drow(node)[row] = 1;
        }
        goto after_value;
      }
      if (c == 't' || c == 'f') {
        const int64_t s = r.p;
        const bool v = (c == 't');
        if (!take_literal(r, c)) break;
        if (t == FT_BOOL) {
          a.vrow(vs)[row] = v ? 1 : 0;
          a.drow(node)[row] = 1;
        } else if (t == FT_STRING) {
          a.vrow(vs)[row] = s;
          a.lrow(ls)[row] = v ? 4 : 5;
          a.drow(node)[row] = 1;
        }
        goto after_value;
      }
      if (c == 'n') {
        if (!take_literal(r, c)) break;
        goto after_value;
      }
      break;  // unexpected token
    }
    // the one place a value is skipped (unknown key, raw-JSON container, too-deep struct): a single inlined copy of
    // the validating skipper keeps the loop's code and register footprint small
  skip_any: {
      const int64_t s0 = r.p;
      if (c == '-' || is_digit(c)) {                       // scalars without the container state machine
        if (!skip_number(r, c, nextc)) break;
      } else if (c == '"') {
        int64_t s, e;
        bool esc;
        if (!scan_string(r, s, e, esc, nextc)) break;
      } else if (!skip_value(r)) {
        break;
      }
      if (store_node >= 0) {
        a.vrow(tb.val_slot[store_node])[row] = s0;
        a.lrow(tb.len_slot[store_node])[row] = (int32_t)(r.p - s0);
        a.drow(store_node)[row] = 1;
      }
    }
  after_value:
    c = (nextc == 256u || nextc == ' ' || nextc == '\n' || nextc == '\r' || nextc == '\t') ? r.ws_cur() : nextc;
    if (c == ',') { ++r.p; comma = true; continue; }
    if (c == '}') continue;  // closes the current object at loop top
    break;
  }
  if (ok) {                   // nothing but whitespace may follow the record's object
    r.skip_ws();
    ok = r.p >= r.end;
  }
done:
  a.row_ok[row] = ok ? 1 : 0;
  if (!ok) {
    for (int k = 0; k < a.nnodes; ++k) a.drow(k)[row] = 0;
  }
#undef stack
#undef expect
}

// Per-node null counts so the host can drop validity masks of columns that turned out complete — every later
// operator then skips its null handling.  blockIdx.y = node; each lane counts 8 rows from one 8-B word (validity
// bytes are 0/1: nulls = rows - popcount), a wave sums by shuffles and adds once.
__global__ __launch_bounds__(256) void null_count_kernel(const uint8_t* __restrict__ valid, int64_t n,
                                                         unsigned long long* __restrict__ nulls) {
  const int k = blockIdx.y;
  const int64_t r0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  unsigned long long cnt = 0;
  if (r0 < n) {
    const int32_t avail = n - r0 < 8 ? (int32_t)(n - r0) : 8;
    const uint8_t* p = valid + (int64_t)k * n + r0;
    const uintptr_t x = reinterpret_cast<uintptr_t>(p);
    const int m = (int)(x & 7);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(x - m);
    uint64_t v = q[0] >> (8 * m);
    if (m && 8 - m < avail) v |= q[1] << (64 - 8 * m);
    if (avail < 8) v &= (1ull << (8 * avail)) - 1;
    cnt = (unsigned long long)(avail - __popcll(v & 0x0101010101010101ull));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(&nulls[k], cnt);
}

// Newline framing: offsets of '\n'-terminated records in a raw byte stream (blob / socket / LZ4-lines sources).
// One wave owns a segment and streams it in coalesced 1 KiB steps (16 B per lane); newline bytes are found with
// an exact SWAR zero-byte test, counted with popcount, and (write pass) placed with a wave prefix sum.
__device__ __forceinline__ uint64_t nl_bytes(uint64_t x) {
  const uint64_t t = x ^ 0x0a0a0a0a0a0a0a0aull;
  const uint64_t y = ((t & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | t;
  return ~y & 0x8080808080808080ull;                    // bit 7 of byte j set iff byte j == '\n'
}

__device__ __forceinline__ void nl_masks(const uint8_t* buf, int64_t p, int64_t end, uint64_t& m0, uint64_t& m1) {
  m0 = m1 = 0;
  if (p >= end) return;
  const uint4 v = *reinterpret_cast<const uint4*>(buf + p);
  m0 = nl_bytes(((uint64_t)v.y << 32) | v.x);
  m1 = nl_bytes(((uint64_t)v.w << 32) | v.z);
  const int64_t rem = end - p;
  if (rem < 16) {
    if (rem <= 8) { m1 = 0; if (rem < 8) m0 &= (1ull << (8 * rem)) - 1; }
    else m1 &= (1ull << (8 * (rem - 8))) - 1;
  }
}

// bit 7 of each byte (nl_bytes) → bit j = byte j
__device__ __forceinline__ uint32_t nl_pack8(uint64_t m) { return (uint32_t)(((m >> 7) * 0x0102040810204080ull) >> 56); }

// Count pass.  With `bits` it also stores each lane's 16-byte newline mask as 16 bits (1/8 of the input), so the
// write pass reads the masks instead of the text a second time.
__global__ __launch_bounds__(256) void count_newlines_kernel(const uint8_t* __restrict__ buf, int64_t len,
                                                             int64_t seg, int64_t nseg,
                                                             int64_t* __restrict__ counts,
                                                             uint16_t* __restrict__ bits) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;                                   // whole waves exit together
  const int64_t beg = s * seg;
  const int64_t end = beg + seg < len ? beg + seg : len;
  uint32_t c = 0;
  for (int64_t p = beg + lane * 16; p < end; p += 1024) {
    uint64_t m0, m1;
    nl_masks(buf, p, end, m0, m1);
    c += __popcll(m0) + __popcll(m1);
    if (bits) bits[p >> 4] = (uint16_t)(nl_pack8(m0) | (nl_pack8(m1) << 8));
  }
  for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) counts[s] = c;
}

// Write pass over the packed masks: `pos[k] = position of the k-th newline + delta`.
__global__ __launch_bounds__(256) void write_newlines_bits_kernel(const uint16_t* __restrict__ bits, int64_t len,
                                                                  int64_t seg, int64_t nseg,
                                                                  const int64_t* __restrict__ base,
                                                                  int64_t* __restrict__ pos, int64_t cap,
                                                                  int64_t delta) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nseg) return;
  const int64_t beg = s * seg;
  const int64_t end = beg + seg < len ? beg + seg : len;
  int64_t k = base[s];
  for (int64_t it = beg; it < end; it += 1024) {           // uniform trip count: shuffles see the whole wave
    const int64_t p = it + lane * 16;
    uint32_t m = p < end ? bits[p >> 4] : 0u;
    const uint32_t c = __popc(m);
    uint32_t incl = c;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    int64_t q = k + (incl - c);
    while (m) { const int j = __builtin_ctz(m); if (q < cap) pos[q] = p + j + delta; ++q; m &= m - 1; }
    k += __shfl(incl, 63, 64);
  }
}

// Zero `nbytes` at `p` with 16-byte stores: the validity planes' clear as a kernel of the parse library.  On an idle
// GPU it and hipMemsetAsync both clear a 33 MB plane in ~6.8 us (tools/gpu/zero_probe.hip); inside the flows either
// one's duration is inflated by the kernels other streams run meanwhile (profiles/round6/parse/README.md).  Head /
// tail bytes outside the aligned body are stored singly.
__global__ void zero_bytes_kernel(uint8_t* __restrict__ p, int64_t nbytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const int64_t head = (int64_t)((16 - (a & 15)) & 15) < nbytes ? (int64_t)((16 - (a & 15)) & 15) : nbytes;
  const int64_t body = (nbytes - head) / 16;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (int64_t i = tid; i < body; i += stride) q[i] = make_uint4(0, 0, 0, 0);
  const int64_t tail0 = head + body * 16;
  if (tid < head) p[tid] = 0;
  if (tid < nbytes - tail0) p[tail0 + tid] = 0;
}

hipError_t zero_bytes(uint8_t* p, int64_t nbytes, hipStream_t s) {
  if (nbytes <= 0) return hipSuccess;
  const int64_t body = nbytes / 16 + 1;
  const int64_t blocks = (body + 255) / 256 < 4096 ? (body + 255) / 256 : 4096;
  hipLaunchKernelGGL(zero_bytes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, nbytes);
  return hipGetLastError();
}

}  // namespace

DXA_API int dxa_json_parse(uint8_t* buf, const int64_t* offs, int64_t n, const uint64_t* lut_keys,
                           const int32_t* lut_node, int32_t lut_cap, const int32_t* node_type,
                           const int32_t* val_slot, const int32_t* len_slot, int32_t nnodes, int64_t* vals,
                           int32_t* lens, uint8_t* valid, uint8_t* row_ok, const int32_t* first_child,
                           const int32_t* next_sib, const int32_t* key_word, const int32_t* key_len,
                           const uint64_t* key_words, int32_t nkey_words, const int64_t* ends, int64_t* vals2,
                           int32_t* lens2, uint8_t* valid2, int32_t nkv, int32_t nkl, int32_t nkn,
                           const int32_t* zslots, int32_t nz, void* stream) {
  if (n <= 0) return 0;
  if (nnodes >= 32767) return (int)hipErrorInvalidValue;   // node ids live in 16-bit LDS nesting slots
  if (nkn < 1 || nkn > nnodes) return (int)hipErrorInvalidValue;
  ParseArgs a{buf, offs, n, lut_keys, lut_node, lut_cap, node_type, val_slot, len_slot, nnodes, vals, lens,
              valid, row_ok, first_child, next_sib, key_word, key_len, key_words, nkey_words, ends, vals2, lens2,
              valid2, nkv, nkl, nkn, zslots, nz};
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = zero_bytes(valid, (int64_t)nkn * n, s);
  if (e != hipSuccess) return (int)e;
  if (nnodes > nkn) {
    e = zero_bytes(valid2, (int64_t)(nnodes - nkn) * n, s);
    if (e != hipSuccess) return (int)e;
  }
  const int block = 256;
  const int64_t grid = (n + block - 1) / block;
  const int64_t tab_bytes = tables_lds_bytes(nnodes, nkey_words, lut_cap);
  if (tab_bytes <= 24 * 1024)
    hipLaunchKernelGGL(json_parse_kernel<true>, dim3((unsigned)grid), dim3(block), (size_t)tab_bytes, s, a);
  else
    hipLaunchKernelGGL(json_parse_kernel<false>, dim3((unsigned)grid), dim3(block), 0, s, a);
  return (int)hipGetLastError();
}

DXA_API int dxa_null_counts(const uint8_t* valid, int64_t n, int32_t nnodes, unsigned long long* nulls, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(nulls, 0, sizeof(unsigned long long) * (size_t)nnodes, s);
  if (e != hipSuccess) return (int)e;
  if (n <= 0 || nnodes <= 0) return 0;
  hipLaunchKernelGGL(null_count_kernel, dim3((unsigned)((n + 2047) / 2048), (unsigned)nnodes), dim3(256), 0, s, valid, n,
                     nulls);
  return (int)hipGetLastError();
}

DXA_API int dxa_count_newlines(const uint8_t* buf, int64_t len, int64_t seg, int64_t* counts, uint16_t* bits,
                               void* stream) {
  if (len <= 0) return 0;
  if (((uintptr_t)buf & 15) || (seg & 1023)) return (int)hipErrorInvalidValue;
  const int64_t nseg = (len + seg - 1) / seg;
  hipLaunchKernelGGL(count_newlines_kernel, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, (hipStream_t)stream, buf,
                     len, seg, nseg, counts, bits);
  return (int)hipGetLastError();
}

// `bits` from dxa_count_newlines (same len / seg); writes newline position + delta
DXA_API int dxa_write_newlines_bits(const uint16_t* bits, int64_t len, int64_t seg, const int64_t* base, int64_t* pos,
                                    int64_t cap, int64_t delta, void* stream) {
  if (len <= 0) return 0;
  if (seg & 1023) return (int)hipErrorInvalidValue;
  const int64_t nseg = (len + seg - 1) / seg;
  hipLaunchKernelGGL(write_newlines_bits_kernel, dim3((unsigned)((nseg + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     bits, len, seg, nseg, base, pos, cap, delta);
  return (int)hipGetLastError();
}
