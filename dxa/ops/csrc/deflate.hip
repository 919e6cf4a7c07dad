// gzip on the device for blob sinks (the reference's GZipHelper.deflateToBytes, K23 in SURVEY §2.F).
//
// The serialized JSON is cut into fixed-size chunks; every chunk becomes one complete gzip member (RFC 1952: a
// 10-byte header, one final deflate block with the fixed Huffman code, CRC-32, ISIZE), so the members need no
// coordination and their concatenation is a valid multi-member gzip file (gunzip / zlib with auto-detect / Python's
// gzip all read it).  One wave owns one chunk, staged in LDS (see gzip_chunks_kernel):
//   * LZ77 over a 4-byte hash (2048 uint16 heads in LDS), greedy parsing — JSON lines repeat their keys and structure,
//     which is where deflate's gain comes from;
//   * the fixed Huffman code (RFC 1951 §3.2.6), token bits placed by a wave prefix sum;
//   * CRC-32 per lane slice, combined across the wave with the GF(2) multiply of crc32_combine.
// A second kernel packs the members back to back (exclusive scan of their sizes on the host side).
// Dynamic Huffman tables would gain more ratio; the fixed code keeps the encoder to one pass, and the output D2H
// (what this is for: PCIe, not HBM, is the bound) is already cut ~5-6x on the serialized events.
#include "dxa_common.h"

namespace {

constexpr int kHashBits = 11;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kMaxDist = 32768;
constexpr int kHdr = 12;             // slot layout: [2 pad][10 gzip header][deflate …][crc32][isize]

__device__ __forceinline__ uint32_t rev_bits(uint32_t code, int len) { return __builtin_bitreverse32(code) >> (32 - len); }

// ---- CRC-32 pieces (reflected polynomial 0xEDB88320) ----------------------------------------------------------
// a·b mod P in the reflected bit order (x^0 is the top bit): the multiply that crc32_combine is built on —
// crc(A‖B) = (crc(A) · x^(8|B|)) ⊕ crc(B).  Lanes CRC their own slices and the wave combines them in a tree.
__host__ __device__ constexpr uint32_t mulmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m != 0; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? ((b >> 1) ^ 0xEDB88320u) : (b >> 1);
  }
  return p;
}

struct X2N {                          // v[k] = x^(2^k) mod P
  uint32_t v[32];
  constexpr X2N() : v{} {
    uint32_t p = 1u << 30;            // x^1
    for (int k = 0; k < 32; ++k) { v[k] = p; p = mulmodp(p, p); }
  }
};
__constant__ X2N kX2N = X2N();

// x^(8n) mod P
__device__ __forceinline__ uint32_t x8n(uint32_t n) {
  uint32_t p = 1u << 31;              // x^0
  for (int k = 3; n != 0; n >>= 1, ++k)
    if (n & 1) p = mulmodp(kX2N.v[k & 31], p);
  return p;
}

struct CrcPow {
  int32_t slice;                      // bytes per lane slice (a multiple of 4, an odd number of words)
  uint32_t x[6];                      // x^(8·slice·2^l) mod P
};

uint32_t host_x8n(uint64_t n) {
  constexpr X2N t{};
  uint32_t p = 1u << 31;
  for (int k = 3; n != 0; n >>= 1, ++k)
    if (n & 1) p = mulmodp(t.v[k & 31], p);
  return p;
}

__device__ __forceinline__ uint32_t lds_load4(const uint32_t* w, int32_t p) {
  const uint32_t a = w[p >> 2], b = w[(p >> 2) + 1];
  const int sh = (p & 3) * 8;
  return sh ? ((a >> sh) | (b << (32 - sh))) : a;
}

// deflate length / distance symbols (RFC 1951 §3.2.5): symbol, extra-bit count, extra-bit value
__device__ __forceinline__ void len_sym(int32_t len, uint32_t& sym, uint32_t& eb, uint32_t& ev) {
  const uint32_t x = (uint32_t)(len - 3);
  eb = 0; ev = 0;
  if (len == 258) sym = 285;
  else if (x < 8) sym = 257 + x;
  else { const int hb = 31 - __builtin_clz(x); eb = hb - 2; sym = 257 + 4 * (hb - 1) + ((x >> eb) & 3); ev = x & ((1u << eb) - 1); }
}
__device__ __forceinline__ void dist_sym(int32_t dist, uint32_t& dc, uint32_t& eb, uint32_t& ev) {
  const uint32_t y = (uint32_t)(dist - 1);
  eb = 0; ev = 0;
  if (y < 4) dc = y;
  else { const int hb = 31 - __builtin_clz(y); eb = hb - 1; dc = 2 * hb + ((y >> eb) & 1); ev = y & ((1u << eb) - 1); }
}

// fixed Huffman literal/length code (RFC 1951 §3.2.6): bit-reversed code | length << 16
__device__ __forceinline__ uint32_t fixed_code(uint32_t sym) {
  if (sym < 144) return rev_bits(0x30 + sym, 8) | (8u << 16);
  if (sym < 256) return rev_bits(0x190 + (sym - 144), 9) | (9u << 16);
  if (sym < 280) return rev_bits(sym - 256, 7) | (7u << 16);
  return rev_bits(0xC0 + (sym - 280), 8) | (8u << 16);
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

constexpr int kRing = 128;            // output word ring (one emit round writes ≤ 97 words)
constexpr int kNLL = 286, kND = 30, kDOff = 288, kNSym = 320;   // LL alphabet at 0 (288 slots: the fixed code
                                                                // defines 286/287), distances at kDOff

struct Out {                          // the chunk's deflate bit stream: LDS word ring → slot words
  uint32_t* win;
  uint32_t* dst;
  uint32_t gbit = 0;                  // bits emitted
  int32_t wbase = 0;                  // first word not yet flushed

  __device__ __forceinline__ void place(uint32_t v, uint32_t n, uint32_t pos) {
    if (!n) return;
    const uint32_t wi = pos >> 5, sh = pos & 31;
    atomicOr(&win[wi & (kRing - 1)], v << sh);
    if (sh && sh + n > 32) atomicOr(&win[(wi + 1) & (kRing - 1)], v >> (32 - sh));
  }
  // every lane appends (a: na bits, then b: nb bits), lanes in order; na, nb ≤ 28.  Offsets by a prefix sum over
  // six bit planes of na + nb (ballots + mbcnt); complete words leave for the slot (a wave's LDS operations
  // complete in order, so the ORs are visible to the flush reads without a barrier)
  __device__ __forceinline__ void emit(uint32_t a, uint32_t na, uint32_t b, uint32_t nb, int lane) {
    const uint32_t n = na + nb;
    uint32_t excl = 0, total = 0;
    for (int bp = 0; bp < 6; ++bp) {
      const uint64_t m = __ballot((n >> bp) & 1);
      excl += lanes_below(m) << bp;
      total += (uint32_t)__builtin_popcountll(m) << bp;
    }
    place(a, na, gbit + excl);
    place(b, nb, gbit + excl + na);
    gbit += total;
    __builtin_amdgcn_wave_barrier();
    const int32_t nfull = (int32_t)(gbit >> 5) - wbase;
    for (int k = lane; k < nfull; k += 64) {
      const int idx = (wbase + k) & (kRing - 1);
      dst[wbase + k] = win[idx];
      win[idx] = 0;
    }
    wbase += nfull;
    __builtin_amdgcn_wave_barrier();
  }
};

// One 64-position group of the greedy LZ77 parse (identical in both passes): every lane hashes its position and
// looks up the newest earlier position with that hash (heads from earlier groups); a candidate is checked for its
// first 4 bytes; the walk takes a literal run up to the next match start in one step and measures that match with
// the whole wave (64 lanes × 4 bytes = 256 bytes per step).  Returns this lane's token: 0 none, 1 literal, 2 match.
__device__ __forceinline__ int parse_group(const uint32_t* dat32, uint16_t* head, int32_t L, int32_t g,
                                           int32_t& carry, int lane, uint32_t& lit, int32_t& len, int32_t& dist) {
  const int32_t p = g + lane;
  const bool can = p + 4 <= L;
  const uint32_t v = lds_load4(dat32, p);
  const uint32_t h = (v * 2654435761u) >> (32 - kHashBits);
  const int32_t cand = can ? (int32_t)head[h] - 1 : -1;
  __builtin_amdgcn_wave_barrier();
  if (can) head[h] = (uint16_t)(p + 1);     // lanes sharing a hash: one of them wins (a candidate, not the newest)
  const bool is_m = cand >= 0 && p - cand <= kMaxDist && lds_load4(dat32, cand) == v;
  const uint64_t mm = __ballot(is_m);
  const uint64_t live = (L - g) >= 64 ? ~0ull : ((1ull << (L - g)) - 1);
  uint64_t tok = 0;
  len = 0;
  int32_t w = carry;
  while (w < 64) {
    const uint64_t from = ~0ull << w;
    const uint64_t rest = mm & from;
    if (rest == 0) { tok |= from; w = 64; break; }
    const int m = __builtin_ctzll(rest);
    tok |= (from & ~(~0ull << m)) | (1ull << m);
    const int32_t pm = g + m, cm = __builtin_amdgcn_readlane(cand, m);
    const int32_t lim = (L - pm) < 258 ? (L - pm) : 258;
    const int32_t off = 4 + 4 * lane;
    const uint32_t x = off < lim ? (lds_load4(dat32, cm + off) ^ lds_load4(dat32, pm + off)) : 0u;
    const uint64_t miss = __ballot(x != 0);
    int32_t ml = lim;
    if (miss) {
      const int k0 = __builtin_ctzll(miss);
      const int32_t e = 4 + 4 * k0 + (__builtin_ctz(__builtin_amdgcn_readlane(x, k0)) >> 3);
      ml = e < lim ? e : lim;
    }
    if (lane == m) len = ml;
    w = m + ml;
  }
  carry = w - 64;
  tok &= live;
  lit = v & 0xff;
  dist = p - cand;
  if (!((tok >> lane) & 1)) return 0;
  return len >= 4 ? 2 : 1;
}

// Code lengths for n symbols from their counts, limited to 15 bits, as a complete prefix code (what inflate
// accepts; a single used symbol gets length 1 — the one incomplete code it allows).  Shannon lengths
// ceil(log2(total/f)), then an over-full Kraft sum is repaired by lengthening the longest codes below 15, and the
// slack is filled by shortening the longest codes (the slack is always a multiple of their Kraft weight).
// Returns the Kraft sum in units of 2^-15.
__device__ uint32_t build_lengths(const uint32_t* hist, uint32_t* lens, int n, int lane) {
  uint32_t tot = 0;
  for (int i = lane; i < n; i += 64) tot += hist[i];
  tot = wave_sum(tot);
  uint32_t kr = 0;
  for (int i = lane; i < n; i += 64) {
    const uint32_t f = hist[i];
    uint32_t l = 0;
    if (f) {
      const float r = __log2f((float)tot / (float)f);
      l = (uint32_t)ceilf(r);
      l = l < 1 ? 1 : (l > 15 ? 15 : l);
      kr += 1u << (15 - l);
    }
    lens[i] = l;
  }
  uint32_t K = wave_sum(kr);
  for (int l = 14; l >= 1 && K > 32768u; --l) {
    const uint32_t need = (K - 32768u + (1u << (14 - l)) - 1) >> (14 - l);
    uint32_t seen = 0;
    for (int r = 0; r < n && seen < need; r += 64) {
      const int i = r + lane;
      const bool at = i < n && lens[i] == (uint32_t)l;
      const uint64_t m = __ballot(at);
      if (at && seen + lanes_below(m) < need) lens[i] = l + 1;
      seen += (uint32_t)__builtin_popcountll(m);
    }
    K -= (seen < need ? seen : need) << (14 - l);
  }
  for (int l = 15; l >= 2 && K < 32768u; --l) {
    const uint32_t need = (32768u - K) >> (15 - l);
    uint32_t seen = 0;
    for (int r = 0; r < n && seen < need; r += 64) {
      const int i = r + lane;
      const bool at = i < n && lens[i] == (uint32_t)l;
      const uint64_t m = __ballot(at);
      if (at && seen + lanes_below(m) < need) lens[i] = l - 1;
      seen += (uint32_t)__builtin_popcountll(m);
    }
    K += (seen < need ? seen : need) << (15 - l);
  }
  __builtin_amdgcn_wave_barrier();
  return K;
}

// Canonical codes (RFC 1951 §3.2.2) for n lengths → tab[i] = bit-reversed code | length << 16.  nc: 16 LDS words.
__device__ void assign_codes(const uint32_t* lens, uint32_t* tab, int n, uint32_t* nc, int lane) {
  uint32_t cnt = 0;                   // lane l (1..15) counts the codes of length l
  for (int i = 0; i < n; ++i) cnt += (lane >= 1 && lane <= 15 && lens[i] == (uint32_t)lane) ? 1u : 0u;
  // next_code[l] = (next_code[l-1] + count[l-1]) << 1
  uint32_t code = 0;
  for (int l = 1; l <= 15; ++l) {
    const uint32_t prev = __shfl(cnt, l - 1, 64);
    code = (code + (l >= 2 ? prev : 0u)) << 1;
    if (lane == l) nc[l] = code;
  }
  __builtin_amdgcn_wave_barrier();
  for (int r = 0; r < n; r += 64) {
    const int i = r + lane;
    const uint32_t l = i < n ? lens[i] : 0u;
    uint32_t c = 0;
    for (int ll = 1; ll <= 15; ++ll) {
      const uint64_t m = __ballot(l == (uint32_t)ll);
      if (!m) continue;
      if (l == (uint32_t)ll) c = nc[ll] + lanes_below(m);
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) nc[ll] += (uint32_t)__builtin_popcountll(m);
      __builtin_amdgcn_wave_barrier();
    }
    if (i < n) tab[i] = l ? (rev_bits(c, (int)l) | (l << 16)) : 0u;
  }
  __builtin_amdgcn_wave_barrier();
}

// One wave per chunk, everything in LDS: [chunk bytes + pad][hash heads][output word window].
//   per 64-position group: every lane hashes its position and looks up the newest earlier position with that
//   hash (heads from earlier groups), extends the match 4 bytes at a time;
//   the greedy parse walks the group with ballots (a literal run up to the next match start in one step);
//   token codes are placed with a wave prefix sum of their bit lengths and OR-ed into the word window, whose
//   complete words go to the chunk's slot after every group.

template <bool kDyn>
__global__ void __launch_bounds__(64) gzip_chunks_kernel(const uint8_t* __restrict__ in, int64_t n_in, int32_t chunk,
                                                         int64_t n_chunks, uint8_t* __restrict__ slots,
                                                         int64_t slot_bytes, int32_t* __restrict__ out_len,
                                                         CrcPow pw, uint32_t* __restrict__ toks) {
  extern __shared__ uint32_t gz_sh[];
  __shared__ uint32_t crc_tab[256];
  const int lane = threadIdx.x;
  for (int k = lane; k < 256; k += 64) {
    uint32_t c = (uint32_t)k;
    for (int j = 0; j < 8; ++j) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    crc_tab[k] = c;
  }
  uint32_t* dat32 = gz_sh;
  const uint8_t* dat = (const uint8_t*)gz_sh;
  uint16_t* head = (uint16_t*)(gz_sh + (chunk >> 2) + 4);     // newest position + 1 per hash (0: none)
  uint32_t* win = gz_sh + (chunk >> 2) + 4 + kHashSize / 2;
  const int64_t c = blockIdx.x;
  const int64_t base = c * chunk;
  const int32_t L = (int32_t)((n_in - base) < chunk ? (n_in - base) : chunk);
  const uint8_t* src = in + base;
  uint8_t* slot = slots + c * slot_bytes;
  uint32_t* dst = (uint32_t*)(slot + kHdr);

  // stage the chunk (16-byte loads; the chunk start is 16-byte aligned), zero the pad, clear the heads
  const int32_t L16 = L & ~15;
  for (int32_t k = lane * 16; k < L16; k += 64 * 16) {
    const uint4 q = *(const uint4*)(src + k);
    dat32[(k >> 2) + 0] = q.x; dat32[(k >> 2) + 1] = q.y; dat32[(k >> 2) + 2] = q.z; dat32[(k >> 2) + 3] = q.w;
  }
  for (int32_t k = L16 + lane; k < ((L + 3) & ~3) + 16; k += 64) {
    // the words past L16: assembled from bytes (zero beyond L)
    if ((k & 3) == 0) {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) if (k + b < L) w |= (uint32_t)src[k + b] << (8 * b);
      dat32[k >> 2] = w;
    }
  }
  for (int k = lane; k < kHashSize / 2; k += 64) gz_sh[(chunk >> 2) + 4 + k] = 0;
  for (int k = lane; k < kRing; k += 64) win[k] = 0;
  if (lane < 10) {
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 0xff};
    slot[2 + lane] = hdr[lane];
  }
  __syncthreads();

  // CRC-32: 64 slices (an odd number of words each, so the lanes' word reads fall in distinct LDS banks), then a
  // tree of combines; the x^(8·len) multipliers of full slices come precomputed from the host
  const int32_t S = pw.slice;
  const int32_t s0 = lane * S < L ? lane * S : L;
  const int32_t s1 = s0 + S < L ? s0 + S : L;
  uint32_t crc = 0xFFFFFFFFu;
  int32_t k = s0;
  for (; k + 4 <= s1; k += 4) {
    const uint32_t w = dat32[k >> 2];
    crc = crc_tab[(crc ^ w) & 0xff] ^ (crc >> 8);
    crc = crc_tab[(crc ^ (w >> 8)) & 0xff] ^ (crc >> 8);
    crc = crc_tab[(crc ^ (w >> 16)) & 0xff] ^ (crc >> 8);
    crc = crc_tab[(crc ^ (w >> 24)) & 0xff] ^ (crc >> 8);
  }
  for (; k < s1; ++k) crc = crc_tab[(crc ^ dat[k]) & 0xff] ^ (crc >> 8);
  crc ^= 0xFFFFFFFFu;
  if (s1 == s0) crc = 0;
  uint32_t clen = (uint32_t)(s1 - s0);
  for (int l = 0; l < 6; ++l) {
    const int d = 1 << l;
    const uint32_t ocrc = __shfl_down(crc, d, 64), olen = __shfl_down(clen, d, 64);
    if ((lane & (2 * d - 1)) == 0 && olen != 0) {
      crc = mulmodp(olen == (uint32_t)(S << l) ? pw.x[l] : x8n(olen), crc) ^ ocrc;
      clen += olen;
    }
  }
  crc = __shfl(crc, 0, 64);

  uint32_t* hist = win + kRing;       // [kNSym] counts: LL at 0, D at kDOff (dynamic only)
  uint32_t* lens = hist + kNSym;      // [kNSym] code lengths
  uint32_t* tab = lens + kNSym;       // [kNSym] codes
  uint32_t* nc = tab + kNSym;         // [16]
  bool use_dyn = false;
  uint32_t nll = 257, ndist = 1;
  int32_t carry = 0;                  // how far the previous group's last match reaches into this group
  if constexpr (kDyn) {
    // pass 1: parse, count symbols
    for (int k = lane; k < kNSym; k += 64) hist[k] = 0;
    __syncthreads();
    uint32_t* tk = toks + c * chunk;
    for (int32_t g = 0; g < L; g += 64) {
      uint32_t lit; int32_t len, dist;
      const int t = parse_group(dat32, head, L, g, carry, lane, lit, len, dist);
      // the parse, kept for pass 2 (coalesced, 256 B per group): type << 30 | literal, or len << 15 | dist
      if (g + lane < L)
        tk[g + lane] = t == 1 ? (1u << 30) | lit : t == 2 ? (2u << 30) | ((uint32_t)len << 15) | (uint32_t)dist : 0u;
      if (t == 1) {
        atomicAdd(&hist[lit], 1u);
      } else if (t == 2) {
        uint32_t sym, eb, ev, dc, deb, dev;
        len_sym(len, sym, eb, ev);
        dist_sym(dist, dc, deb, dev);
        atomicAdd(&hist[sym], 1u);
        atomicAdd(&hist[kDOff + dc], 1u);
      }
    }
    if (lane == 0) hist[256] += 1;      // end of block
    for (int k = lane; k < kHashSize / 2; k += 64) gz_sh[(chunk >> 2) + 4 + k] = 0;
    __syncthreads();

    // dynamic code lengths; the block is written with them only when that (header included) beats the fixed code
    // (the extra bits of lengths and distances are the same either way)
    for (int k = lane; k < kNSym; k += 64) lens[k] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t k_ll = build_lengths(hist, lens, kNLL, lane);
    const uint32_t k_d = build_lengths(hist + kDOff, lens + kDOff, kND, lane);
    const uint64_t used_d = __ballot(lane < kND && lens[kDOff + lane] != 0);
    if (used_d == 0 && lane == 0) lens[kDOff] = 1;                         // no match: one (unused) distance code
    const bool single_d = __builtin_popcountll(used_d) <= 1;
    uint32_t hi_ll = 0;
    for (int i = lane; i < kNLL; i += 64) if (lens[i]) hi_ll = i;
    for (int d = 32; d >= 1; d >>= 1) { const uint32_t o = __shfl_xor(hi_ll, d, 64); hi_ll = o > hi_ll ? o : hi_ll; }
    nll = hi_ll + 1 < 257 ? 257 : hi_ll + 1;
    ndist = used_d ? 64 - __builtin_clzll(used_d) : 1;
    uint32_t dyn = 0, fix = 0;
    for (int i = lane; i < kNSym; i += 64) {
      const uint32_t f = hist[i];
      const uint32_t fl = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < kDOff ? 8 : 5;
      dyn += f * lens[i];
      fix += f * fl;
    }
    dyn = wave_sum(dyn) + 17 + 57 + 4 * (nll + ndist);
    fix = wave_sum(fix);
    use_dyn = k_ll == 32768u && (k_d == 32768u || single_d) && dyn < fix;
    __syncthreads();
    if (!use_dyn)
      for (int i = lane; i < kNSym; i += 64)
        lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < kDOff ? 8 : (i < kDOff + kND ? 5 : 0);
    __syncthreads();
    assign_codes(lens, tab, kDOff, nc, lane);
    for (int k = lane; k < 16; k += 64) nc[k] = 0;
    __syncthreads();
    assign_codes(lens + kDOff, tab + kDOff, kND, nc, lane);
    __syncthreads();


  }
  Out o;
  o.win = win;
  o.dst = dst;
  if (use_dyn) {
    // BFINAL, BTYPE = 10, HLIT, HDIST, HCLEN = 15 (all 19 code-length code lengths follow); the code-length code
    // gives symbols 0..15 four bits each (complete) and RLE symbols 16-18 none
    constexpr uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t a = 0, na = 0;
    if (lane == 0) { a = 1u | (2u << 1) | ((nll - 257) << 3) | ((ndist - 1) << 8) | (15u << 13); na = 17; }
    else if (lane <= 19) { a = kOrder[lane - 1] <= 15 ? 4u : 0u; na = 3; }
    o.emit(a, na, 0, 0, lane);
    for (uint32_t r = 0; r < nll + ndist; r += 64) {
      const uint32_t i = r + lane;
      uint32_t v = 0, nv = 0;
      if (i < nll + ndist) { v = rev_bits(i < nll ? lens[i] : lens[kDOff + (i - nll)], 4); nv = 4; }
      o.emit(v, nv, 0, 0, lane);
    }
  } else {
    o.emit(lane == 0 ? 3u : 0u, lane == 0 ? 3u : 0u, 0, 0, lane);      // BFINAL, BTYPE = 01
  }

  // pass 2: the parse coded (dynamic: read back from pass 1's tokens instead of parsing again)
  carry = 0;
  for (int32_t g = 0; g < L; g += 64) {
    uint32_t lit = 0; int32_t len = 0, dist = 0;
    int t;
    if constexpr (kDyn) {
      const uint32_t w = g + lane < L ? toks[c * chunk + g + lane] : 0u;
      t = (int)(w >> 30);
      lit = w & 0xffu;
      len = (int32_t)((w >> 15) & 0x1ffu);
      dist = (int32_t)(w & 0x7fffu);
    } else {
      t = parse_group(dat32, head, L, g, carry, lane, lit, len, dist);
    }
    uint32_t a = 0, na = 0, b = 0, nb = 0;
    if (t == 1) {
      const uint32_t e = kDyn ? tab[lit] : fixed_code(lit);
      a = e & 0xffff; na = e >> 16;
    } else if (t == 2) {
      uint32_t sym, eb, ev, dc, deb, dev;
      len_sym(len, sym, eb, ev);
      dist_sym(dist, dc, deb, dev);
      const uint32_t e = kDyn ? tab[sym] : fixed_code(sym), e2 = kDyn ? tab[kDOff + dc] : (rev_bits(dc, 5) | (5u << 16));
      a = (e & 0xffff) | (ev << (e >> 16)); na = (e >> 16) + eb;
      b = (e2 & 0xffff) | (dev << (e2 >> 16)); nb = (e2 >> 16) + deb;
    }
    o.emit(a, na, b, nb, lane);
  }
  {
    const uint32_t e = kDyn ? tab[256] : fixed_code(256);               // end of block
    o.emit(lane == 0 ? (e & 0xffff) : 0u, lane == 0 ? (e >> 16) : 0u, 0, 0, lane);
  }
  // the trailer bytes right after the last deflate byte
  const uint32_t nbytes = (o.gbit + 7) >> 3;          // deflate bytes
  if (lane < 8) {
    const uint32_t val = lane < 4 ? crc : (uint32_t)L;
    const uint32_t byte = (val >> (8 * (lane & 3))) & 0xff;
    const uint32_t at = nbytes + lane;                                  // byte offset in the deflate stream
    atomicOr(&win[(at >> 2) & (kRing - 1)], byte << (8 * (at & 3)));
  }
  __syncthreads();
  const int32_t end_words = (int32_t)((nbytes + 8 + 3) >> 2);
  for (int k = o.wbase + lane; k < end_words; k += 64) dst[k] = win[k & (kRing - 1)];
  if (lane == 0) out_len[c] = (int32_t)(10 + nbytes + 8);
}

// member c: slot bytes [2, 2 + out_len[c]) → out[offs[c] …]; one workgroup per member, 16-byte copies where the
// source and destination alignment allow, bytes otherwise
__global__ void __launch_bounds__(256) gzip_pack_kernel(const uint8_t* __restrict__ slots, int64_t slot_bytes,
                                                        const int32_t* __restrict__ out_len,
                                                        const int64_t* __restrict__ offs, int64_t n_chunks,
                                                        uint8_t* __restrict__ out) {
  for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const uint8_t* s = slots + c * slot_bytes + 2;
    uint8_t* d = out + offs[c];
    const int32_t l = out_len[c];
    for (int32_t k = threadIdx.x; k < l; k += blockDim.x) d[k] = s[k];
  }
}

}  // namespace

DXA_API int64_t dxa_gzip_slot_bytes(int32_t chunk) {
  return ((int64_t)kHdr + ((int64_t)chunk * 9 + 7) / 8 + 32 + 15) & ~(int64_t)15;
}

// dynamic: per-member Huffman tables from a counting pass (the block keeps the fixed code when that is smaller);
// `toks` (n_chunks x chunk words) holds the counting pass's parse, so the coding pass does not parse again.
DXA_API int dxa_gzip_chunks(const uint8_t* in, int64_t n_in, int32_t chunk, uint8_t* slots, int32_t* out_len,
                            int32_t dynamic, uint32_t* toks, void* st) {
  if (n_in <= 0) return 0;
  if (chunk < 64 || chunk > 32768 || (chunk & 63)) return (int)hipErrorInvalidValue;   // deflate window
  if (dynamic && toks == nullptr) return (int)hipErrorInvalidValue;
  const int64_t n_chunks = (n_in + chunk - 1) / chunk;
  const int64_t slot = dxa_gzip_slot_bytes(chunk);
  const size_t lds = ((size_t)(chunk >> 2) + 4 + kHashSize / 2 + kRing + (dynamic ? 3 * kNSym + 16 : 0)) * 4;
  CrcPow pw{};
  int32_t words = ((chunk + 63) / 64 + 3) / 4;
  if ((words & 1) == 0) ++words;
  pw.slice = words * 4;
  for (int l = 0; l < 6; ++l) pw.x[l] = host_x8n((uint64_t)pw.slice << l);
  if (dynamic)
    hipLaunchKernelGGL(gzip_chunks_kernel<true>, dim3((unsigned)n_chunks), dim3(64), lds, (hipStream_t)st, in, n_in,
                       chunk, n_chunks, slots, slot, out_len, pw, toks);
  else
    hipLaunchKernelGGL(gzip_chunks_kernel<false>, dim3((unsigned)n_chunks), dim3(64), lds, (hipStream_t)st, in, n_in,
                       chunk, n_chunks, slots, slot, out_len, pw, (uint32_t*)nullptr);
  return (int)hipGetLastError();
}

DXA_API int dxa_gzip_pack(const uint8_t* slots, int32_t chunk, const int32_t* out_len, const int64_t* offs,
                          int64_t n_chunks, uint8_t* out, void* st) {
  if (n_chunks <= 0) return 0;
  hipLaunchKernelGGL(gzip_pack_kernel, dim3(dxa_blocks(n_chunks, 1, 8192)), dim3(256), 0, (hipStream_t)st, slots,
                     dxa_gzip_slot_bytes(chunk), out_len, offs, n_chunks, out);
  return (int)hipGetLastError();
}
