// Register-packed text emitter shared by the device-side text producers (event generator, JSON serializer).
#pragma once
#include "dxa_common.h"

// Full-word stores are ordinary write-back stores: a record's 16-B words arrive at one 128-B line over several store
// instructions and the L2 merges them into whole-line writes.  Measured and dropped: nontemporal stores (each 16-B
// piece leaves as its own partial-line write: the generator's write pass 1.79 ms per 1 M IoT events vs 0.77 ms,
// tools/gpu/gpu_gen_ab.sh) and LDS-staged 64-B segments per lane (PMC write traffic 1.70 -> 0.72 GB, but the
// kernels are issue-bound and the staging cost VGPRs: gen_write 559 vs 544 us, ser_write 1134 vs 1043 us,
// profiles/pmc/passthrough_r4.md).

namespace dxa {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Low `n` bytes of w (n in 0..8).
__device__ __forceinline__ uint64_t low_bytes(uint64_t w, uint32_t n) {
  return n >= 8 ? w : (w & ((1ull << (8 * n)) - 1ull));
}

// One lane renders one record into [dst, dst + len).  Records are contiguous and disjoint, so every 16-B aligned
// word that lies inside a record belongs to that lane alone: the emitter accumulates bytes in a 16-byte register
// pair (a0, a1) and leaves through one aligned 16-B store per word.  Only the record's first and last partial words
// (shared with the neighbouring records) go out as naturally aligned 1/2/4/8-B pieces, both in `finish()`: the
// first word is parked in registers (h0, h1) when it fills, so the per-byte path holds a single store and the
// piecewise stores are inlined once per kernel, not at every emit site.
//
// The unit of input is a word of up to 8 bytes (`put_word`): literal text arrives as 8-B words read from an
// 8-aligned, zero-padded pool (one load per 8 bytes instead of one byte load per byte), and numbers are formatted
// into words of digits before they are emitted.  The length pass (WRITE = false) only counts.
template <bool WRITE>
struct Emitter {
  uint8_t* wbase;      // 16-B aligned address of the current word
  uint8_t* hbase;      // 16-B aligned address of the first word
  int64_t len;         // bytes emitted so far
  uint32_t lead;       // bytes of the first word that belong to the previous record (dst & 15)
  uint32_t nacc;       // bytes of the current word filled (lead included while on the first word)
  bool first;          // still on the record's first word
  uint64_t a0, a1;     // current word
  uint64_t h0, h1;     // the first word, once full (written by finish)

  __device__ __forceinline__ explicit Emitter(uint8_t* dst)
      : len(0), lead(0), nacc(0), first(true), a0(0), a1(0), h0(0), h1(0) {
    if (WRITE) {
      lead = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 15);
      wbase = hbase = dst - lead;
      nacc = lead;
    } else {
      wbase = hbase = nullptr;
    }
  }

  // bytes [lo, hi) of the word held in (x0, x1), as naturally aligned pieces
  __device__ __forceinline__ static void store_range(uint8_t* w, uint64_t x0, uint64_t x1, uint32_t lo,
                                                     uint32_t hi) {
#pragma unroll 1
    while (lo < hi) {
      const uint64_t src = lo < 8 ? x0 : x1;
      const uint32_t sh = 8 * (lo & 7);
      if ((lo & 7) == 0 && lo + 8 <= hi) {
        *reinterpret_cast<uint64_t*>(w + lo) = src;
        lo += 8;
      } else if ((lo & 3) == 0 && lo + 4 <= hi) {
        *reinterpret_cast<uint32_t*>(w + lo) = (uint32_t)(src >> sh);
        lo += 4;
      } else if ((lo & 1) == 0 && lo + 2 <= hi) {
        *reinterpret_cast<uint16_t*>(w + lo) = (uint16_t)(src >> sh);
        lo += 2;
      } else {
        w[lo] = (uint8_t)(src >> sh);
        lo += 1;
      }
    }
  }

  __device__ __forceinline__ static void store16(uint8_t* w, uint64_t x0, uint64_t x1) {
    u64x2 v;
    v.x = x0;
    v.y = x1;
    *reinterpret_cast<u64x2*>(w) = v;
  }

  __device__ __forceinline__ void flush_full() {
    if (first) {
      h0 = a0;
      h1 = a1;
      first = false;
    } else {
      store16(wbase, a0, a1);
    }
    wbase += 16;
  }

  // Append the low n bytes of w (n in 0..8; bytes of w above n must be zero).
  __device__ __forceinline__ void put_word(uint64_t w, uint32_t n) {
    if (WRITE) {
      const uint32_t sh = 8 * nacc;       // 0..120
      uint64_t ov = 0;
      if (sh < 64) {
        a0 |= w << sh;
        if (sh) a1 |= w >> (64 - sh);
      } else {
        a1 |= w << (sh - 64);
        if (sh > 64) ov = w >> (128 - sh);
      }
      nacc += n;
      if (nacc >= 16) {
        flush_full();
        a0 = ov;
        a1 = 0;
        nacc -= 16;
      }
    }
    len += n;
  }

  __device__ __forceinline__ void put(uint8_t c) { put_word((uint64_t)c, 1); }

  // Literal text from an 8-B aligned, zero-padded pool (`words` is aligned; bytes past n in the last word are 0).
  __device__ __forceinline__ void put_text_words(const uint64_t* words, int32_t n) {
    if (!WRITE) { len += n; return; }
    int32_t q = 0;
    for (; q + 8 <= n; q += 8) put_word(words[q >> 3], 8);
    if (q < n) put_word(words[q >> 3], (uint32_t)(n - q));
  }

  __device__ __forceinline__ void finish() {
    if (WRITE) {
      if (first) {                       // the record never left its first word
        if (nacc > lead) store_range(hbase, a0, a1, lead, nacc);
      } else {
        if (lead == 0) {
          store16(hbase, h0, h1);
        } else {
          store_range(hbase, h0, h1, lead, 16);
        }
        if (nacc) store_range(wbase, a0, a1, 0, nacc);
      }
    }
  }

  // ---- numbers --------------------------------------------------------------------------------------------------
  __device__ __forceinline__ static uint32_t ndigits32(uint32_t x) {
    return 1u + (x >= 10u) + (x >= 100u) + (x >= 1000u) + (x >= 10000u) + (x >= 100000u) + (x >= 1000000u) +
           (x >= 10000000u) + (x >= 100000000u) + (x >= 1000000000u);
  }

  // exactly nd (1..8) digits of x (zero-padded)
  __device__ __forceinline__ void put_fixed(uint32_t x, uint32_t nd) {
    if (!WRITE) { len += nd; return; }
    uint64_t w = 0;
    for (uint32_t i = 0; i < nd; ++i) {        // digit i from the right goes to byte nd-1-i
      const uint32_t q = x / 10u;
      w |= (uint64_t)('0' + (x - q * 10u)) << (8 * (nd - 1 - i));
      x = q;
    }
    put_word(w, nd);
  }

  __device__ __forceinline__ void put_u32(uint32_t x) {
    if (x < 100000000u) {
      put_fixed(x, ndigits32(x));
    } else {
      const uint32_t hi = x / 100000000u;
      put_fixed(hi, ndigits32(hi));
      put_fixed(x - hi * 100000000u, 8);
    }
  }

  __device__ __forceinline__ void put_u64(uint64_t v) {
    if (v <= 0xffffffffull) { put_u32((uint32_t)v); return; }
    const uint64_t hi = v / 100000000ull;
    const uint32_t lo = (uint32_t)(v - hi * 100000000ull);
    if (hi < 100000000ull) {
      put_fixed((uint32_t)hi, ndigits32((uint32_t)hi));
    } else {
      const uint64_t top = hi / 100000000ull;                // < 1845
      put_fixed((uint32_t)top, ndigits32((uint32_t)top));
      put_fixed((uint32_t)(hi - top * 100000000ull), 8);
    }
    put_fixed(lo, 8);
  }

  __device__ __forceinline__ void put_i64(int64_t v) {
    if (v < 0) { put('-'); put_u64(0ull - (uint64_t)v); } else put_u64((uint64_t)v);
  }

  __device__ __forceinline__ void put2(int v) { put_fixed((uint32_t)v, 2); }
};

}  // namespace dxa
