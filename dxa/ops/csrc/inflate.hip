// DEFLATE (RFC 1951) decoder for gfx950: gzip-compressed Kafka record batches (codec 1 — the records section of a
// batch is one gzip member, RFC 1952; the Azure Event Hubs Kafka endpoint's only codec) are decompressed in HBM
// after a compressed H2D copy, like the LZ4 batches (lz4.hip), instead of on the host.
//
// Layout: 16 lanes own one member (the host planner points comp_off at the deflate data after the gzip header and
// takes the decompressed size from the ISIZE trailer).  The Huffman decode is a serial chain, so all 16 lanes run it
// redundantly on wave-uniform-per-group state (64-bit bit buffer refilled with broadcast dword loads); the lanes
// split the work that is parallel: building the decode tables, stored-block copies and match copies.
//   * Decode tables live in LDS, one set per group: a 9-bit fast table for literal/length codes and an 8-bit one for
//     distances ((length << 9) | symbol per entry, built from the canonical code of every symbol no longer than the
//     table index, replicated over the unused high bits by the 16 lanes), plus count / sorted-symbol arrays for the
//     canonical bit-serial path of longer codes (puff's decode).
//   * Matches copy from the block's own output in HBM, 16 bytes per step; a `s_waitcnt vmcnt(0)` before a copy whose
//     source reaches past the bytes known complete makes the group's earlier stores visible (as in lz4.hip).
//   * Every index is bounds-checked: output past the ISIZE capacity, a distance before the output start, a code that
//     is not in the table, over-subscribed code lengths or input past the member end stop the member with a nonzero
//     status (the Kafka source then rejects the batch), never an out-of-range access.
// gzip's CRC-32 of the output is not recomputed here: the batch's CRC-32C (check.crcs) covers the compressed bytes
// in transit, and a corrupt stream fails the decode or the ISIZE check.
#include "dxa_common.h"

namespace {

constexpr int IG = 16;                  // lanes per member
constexpr int WG = 128;                 // threads per workgroup: 8 members
constexpr int LBITS = 9;                // literal/length fast-table bits
constexpr int DBITS = 8;                // distance fast-table bits
constexpr int kWaitVm0 = 0xF70;         // s_waitcnt vmcnt(0) (gfx9 encoding)

// nonzero status = where the member failed (IF_CODE + n: which code check)
enum : int32_t { IF_OK = 0, IF_TRUNC = 1, IF_DIST = 2, IF_OVERFLOW = 3, IF_SIZE = 4, IF_CODE = 10, IF_BLOCK = 6 };

struct Tables {
  uint16_t lfast[1 << LBITS];
  uint16_t dfast[1 << DBITS];
  uint16_t lsorted[288];
  uint16_t dsorted[32];
  uint16_t lcount[16];
  uint16_t dcount[16];
  uint8_t lens[320];                     // code lengths of the block being built (literal/length then distance)
  uint8_t clens[20];                     // code-length code lengths
  uint16_t csorted[19];
  uint16_t ccount[16];                   // build_table writes a count for every length 0..15
};

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                       193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t bitrev(uint32_t c, int n) { return __builtin_bitreverse32(c) >> (32 - n); }

// The 16 lanes of a member hand data to each other through the group's LDS tables (lane 0 writes a code length,
// every lane reads it).  LDS operations of one wave execute in order, but without a fence the compiler may keep or
// move LDS values across the hand-off as if no other lane wrote them — this makes every earlier LDS write of the
// wave visible to every later LDS read (measured: without it, ~1 in 5000 members built its tables from stale LDS).
__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Canonical Huffman tables from code lengths: count per length, symbols sorted by (length, symbol) and (fast != null)
// a `bits`-bit direct table.  Returns false for an over-subscribed set.  All IG lanes call it; lane gl fills every
// IG-th replica of a short code.
__device__ bool build_table(const uint8_t* lens, int n, uint16_t* count, uint16_t* sorted, uint16_t* fast, int bits,
                            int maxlen, int gl) {
  lane_sync();                               // the lengths were written by other lanes of the group
  if (fast) {
    for (int i = gl; i < (1 << bits); i += IG) fast[i] = 0;
    lane_sync();
  }
  uint16_t cnt[16];
  for (int l = 0; l < 16; ++l) cnt[l] = 0;
  for (int s = 0; s < n; ++s) cnt[lens[s]]++;
  int left = 1;
  for (int l = 1; l <= maxlen; ++l) {
    left = (left << 1) - cnt[l];
    if (left < 0) return false;
  }
  uint16_t offs[16];
  offs[1] = 0;
  for (int l = 1; l < 15; ++l) offs[l + 1] = offs[l] + cnt[l];
  if (gl == 0) {
    for (int l = 0; l < 16; ++l) count[l] = cnt[l];
  }
  // canonical first code per length (RFC 1951 3.2.2, zero lengths not counted)
  uint32_t next[16];
  uint32_t code = 0;
  next[0] = 0;
  for (int l = 1; l < 16; ++l) {
    next[l] = code;
    code = (code + cnt[l]) << 1;
  }
  for (int s = 0; s < n; ++s) {
    const int l = lens[s];
    if (!l) continue;
    if (gl == 0) sorted[offs[l]] = (uint16_t)s;
    offs[l]++;
    const uint32_t c = next[l]++;
    if (fast && l <= bits) {
      const uint32_t r = bitrev(c, l);
      const uint16_t e = (uint16_t)((l << 9) | s);
      for (int k = gl; k < (1 << (bits - l)); k += IG) fast[r | ((uint32_t)k << l)] = e;
    }
  }
  lane_sync();                               // tables complete before any lane decodes with them
  return true;
}

__global__ __launch_bounds__(WG) void inflate_group_kernel(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ comp_off,
                                                           const int32_t* __restrict__ comp_len,
                                                           const uint8_t* __restrict__ kind,
                                                           const int64_t* __restrict__ out_off,
                                                           const int64_t* __restrict__ cap_arr, int64_t nb,
                                                           uint8_t* __restrict__ dst, int64_t* __restrict__ produced,
                                                           int32_t* __restrict__ status) {
  __shared__ Tables tabs[WG / IG];
  Tables& T = tabs[threadIdx.x / IG];
  const int64_t b = ((int64_t)blockIdx.x * WG + threadIdx.x) / IG;
  const int gl = (int)(threadIdx.x & (IG - 1));
  if (b >= nb || kind[b] != 2) return;
  const uint8_t* in = src + comp_off[b];
  const int32_t n = comp_len[b];
  const int64_t cap64 = cap_arr[b];
  uint8_t* out = dst + out_off[b];
  if (n < 0 || cap64 < 0 || cap64 > INT32_MAX) {
    if (gl == 0) status[b] = IF_OVERFLOW;
    return;
  }
  const int32_t cap = (int32_t)cap64;
  const int32_t lim = n + 8;             // the 8-byte gzip trailer follows the deflate data: readable
  // ---- bit reader (uniform per group)
  uint64_t bb = 0;
  int bc = 0;
  int32_t ip = 0;
  auto ld32 = [&](int32_t p) -> uint32_t {
    if (p + 4 <= lim) {
      const uintptr_t a = reinterpret_cast<uintptr_t>(in + p);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
      const uint32_t sh = (uint32_t)(a & 3) * 8u;
      const uint32_t lo = w[0];
      if (!sh) return lo;
      return (lo >> sh) | (w[1] << (32u - sh));
    }
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i)
      if (p + i < lim) v |= (uint32_t)in[p + i] << (8 * i);
    return v;
  };
  auto refill = [&]() {
    if (bc <= 32) {
      bb |= (uint64_t)ld32(ip) << bc;
      ip += 4;
      bc += 32;
    }
  };
  auto bits = [&](int k) -> uint32_t {      // k <= 24
    refill();
    const uint32_t v = (uint32_t)(bb & ((1ull << k) - 1));
    bb >>= k;
    bc -= k;
    return v;
  };
  // canonical bit-serial decode of a code longer than the fast table (or with no fast table)
  auto slow = [&](const uint16_t* count, const uint16_t* sorted, int maxlen) -> int {
    refill();
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= maxlen; ++l) {
      code |= (int)(bb & 1);
      bb >>= 1;
      bc--;
      const int c = count[l];
      if (code - first < c) return sorted[index + code - first];
      index += c;
      first = (first + c) << 1;
      code <<= 1;
    }
    return -1;
  };
  auto decode = [&](const uint16_t* fast, int fbits, const uint16_t* count, const uint16_t* sorted) -> int {
    refill();
    const uint32_t e = fast[bb & ((1u << fbits) - 1)];
    const int l = (int)(e >> 9);
    if (l) {
      bb >>= l;
      bc -= l;
      return (int)(e & 511);
    }
    return slow(count, sorted, 15);
  };
  int32_t op = 0, rc = IF_OK, done = 0;
  bool last = false;
  while (!last && rc == IF_OK) {
    if ((int64_t)ip * 8 - bc > (int64_t)lim * 8) { rc = IF_TRUNC; break; }
    last = bits(1) != 0;
    const uint32_t type = bits(2);
    if (type == 0) {                                     // stored block
      const int drop = bc & 7;
      bb >>= drop;
      bc -= drop;
      const uint32_t len = bits(16), nlen = bits(16);
      if ((len ^ 0xffffu) != nlen) { rc = IF_BLOCK; break; }
      const int32_t pos = ip - bc / 8;                   // bytes still buffered are not consumed yet
      if (pos + (int32_t)len > n) { rc = IF_TRUNC; break; }
      if (op + (int32_t)len > cap) { rc = IF_OVERFLOW; break; }
      for (int32_t c = gl; c < (int32_t)len; c += IG) out[op + c] = in[pos + c];
      op += (int32_t)len;
      ip = pos + (int32_t)len;
      bb = 0;
      bc = 0;
      continue;
    }
    if (type == 3) { rc = IF_BLOCK; break; }
    int nlit = 288, ndist = 30;
    if (type == 1) {                                     // fixed codes
      for (int s = gl; s < 320; s += IG) T.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
    } else {                                             // dynamic codes
      nlit = (int)bits(5) + 257;
      ndist = (int)bits(5) + 1;
      const int ncl = (int)bits(4) + 4;
      if (nlit > 286 || ndist > 30) { rc = IF_BLOCK; break; }
      uint32_t cl[19];
      for (int i = 0; i < 19; ++i) cl[i] = 0;
      for (int i = 0; i < ncl; ++i) cl[kClenOrder[i]] = bits(3);
      if (gl == 0) {
        for (int i = 0; i < 19; ++i) T.clens[i] = (uint8_t)cl[i];
      }
      if (!build_table(T.clens, 19, T.ccount, T.csorted, nullptr, 0, 7, gl)) { rc = IF_CODE + 0; break; }
      int i = 0;
      while (i < nlit + ndist) {
        const int sym = slow(T.ccount, T.csorted, 7);
        if (sym < 0) { rc = IF_CODE + 1; break; }
        if (sym < 16) {
          if (gl == 0) T.lens[i] = (uint8_t)sym;
          ++i;
          continue;
        }
        int rep, val = 0;
        if (sym == 16) {
          if (i == 0) { rc = IF_CODE + 2; break; }
          lane_sync();
          val = T.lens[i - 1];
          rep = 3 + (int)bits(2);
        } else if (sym == 17) {
          rep = 3 + (int)bits(3);
        } else {
          rep = 11 + (int)bits(7);
        }
        if (i + rep > nlit + ndist) { rc = IF_CODE + 3; break; }
        for (int k = gl; k < rep; k += IG) T.lens[i + k] = (uint8_t)val;
        i += rep;
      }
      if (rc != IF_OK) break;
      lane_sync();
      if (T.lens[256] == 0) { rc = IF_CODE + 4; break; }   // no end-of-block code
    }
    if (!build_table(T.lens, nlit, T.lcount, T.lsorted, T.lfast, LBITS, 15, gl) ||
        !build_table(T.lens + nlit, ndist, T.dcount, T.dsorted, T.dfast, DBITS, 15, gl)) {
      rc = IF_CODE + 5;
      break;
    }
    // ---- symbols
    for (;;) {
      if ((int64_t)ip * 8 - bc > (int64_t)lim * 8) { rc = IF_TRUNC; break; }
      const int sym = decode(T.lfast, LBITS, T.lcount, T.lsorted);
      if (sym < 0) { rc = IF_CODE + 6; break; }
      if (sym < 256) {
        if (op >= cap) { rc = IF_OVERFLOW; break; }
        if (gl == 0) out[op] = (uint8_t)sym;
        ++op;
        continue;
      }
      if (sym == 256) break;
      const int li = sym - 257;
      if (li >= 29) { rc = IF_CODE + 7; break; }
      const int32_t len = kLenBase[li] + (int32_t)bits(kLenExtra[li]);
      const int ds = decode(T.dfast, DBITS, T.dcount, T.dsorted);
      if (ds < 0 || ds >= 30) { rc = IF_CODE + 8; break; }
      const int32_t dist = kDistBase[ds] + (int32_t)bits(kDistExtra[ds]);
      if (dist > op) { rc = IF_DIST; break; }
      if (len > cap - op) { rc = IF_OVERFLOW; break; }
      const int32_t s0 = op - dist;
      if (s0 + (dist < len ? dist : len) > done) {
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        asm volatile("" ::: "memory");
        done = op;
      }
      if (dist >= len) {
        for (int32_t c = 0; c < len; c += IG)
          if (c + gl < len) out[op + c + gl] = out[s0 + c + gl];
      } else {
        for (int32_t c = 0; c < len; c += IG) {
          const uint32_t k = (uint32_t)(c + gl);
          if ((int32_t)k < len) out[op + (int32_t)k] = out[s0 + (int32_t)(k % (uint32_t)dist)];
        }
      }
      op += len;
    }
  }
  if (rc == IF_OK && op != cap) rc = IF_SIZE;
  if (gl == 0) {
    status[b] = rc;
    produced[b] = op;
  }
}

}  // namespace

// Decode the kind == 2 (deflate) blocks of a Kafka fetch plan: deflate data at comp_off[b] (comp_len[b] bytes, the
// gzip trailer after it), cap[b] = ISIZE bytes reserved at out_off[b]; produced[b] / status[b] out.  Other kinds are
// left to the LZ4 decoder.
DXA_API int dxa_inflate_into(const void* src, const void* comp_off, const void* comp_len, const void* kind,
                             const void* out_off, const void* cap, int64_t nb, void* dst, void* produced, void* status,
                             void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(inflate_group_kernel, dim3((unsigned)((nb * IG + WG - 1) / WG)), dim3(WG), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)kind,
                     (const int64_t*)out_off, (const int64_t*)cap, nb, (uint8_t*)dst, (int64_t*)produced,
                     (int32_t*)status);
  return (int)hipGetLastError();
}
