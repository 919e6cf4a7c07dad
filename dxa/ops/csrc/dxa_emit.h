// Register-packed byte emitter shared by the device-side text producers (event generator, JSON serializer).
#pragma once
#include "dxa_common.h"

namespace dxa {

// Length pass: counts bytes only.  Write pass: bytes are packed into a 16-byte register word and flushed with one
// aligned 16-B store (records are contiguous and disjoint, so every aligned word inside a record belongs to exactly
// one lane); only the unaligned head (< 16 B) and the tail go out as single bytes.  This cuts store instructions
// ~16x versus byte stores — the write pass was store-issue bound (600-B records, one byte per instruction).
template <bool WRITE>
struct Emitter {
  uint8_t* p;
  int64_t len;
  int head;            // leading bytes written singly until p + len is 16-B aligned
  int nacc;            // bytes held in acc
  uint64_t acc0, acc1;

  __device__ __forceinline__ Emitter(uint8_t* dst) : p(dst), len(0), head(0), nacc(0), acc0(0), acc1(0) {
    if (WRITE) head = (int)((16 - ((uintptr_t)dst & 15)) & 15);
  }
  __device__ __forceinline__ void put(uint8_t c) {
    if (WRITE) {
      if (len < head) {
        p[len] = c;
      } else {
        if (nacc < 8) acc0 |= (uint64_t)c << (8 * nacc);
        else acc1 |= (uint64_t)c << (8 * (nacc - 8));
        if (++nacc == 16) {
          uint64_t* w = reinterpret_cast<uint64_t*>(p + len - 15);
          __builtin_nontemporal_store(acc0, w);
          __builtin_nontemporal_store(acc1, w + 1);
          acc0 = acc1 = 0;
          nacc = 0;
        }
      }
    }
    ++len;
  }
  __device__ __forceinline__ void finish() {
    if (WRITE) {
      uint8_t* q = p + len - nacc;
      for (int k = 0; k < nacc; ++k) q[k] = (uint8_t)((k < 8 ? acc0 >> (8 * k) : acc1 >> (8 * (k - 8))) & 0xff);
    }
  }
  __device__ __forceinline__ void put_u64(uint64_t v) {
    char tmp[20];
    int k = 0;
    do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) put((uint8_t)tmp[--k]);
  }
  __device__ __forceinline__ void put_i64(int64_t v) {
    if (v < 0) { put('-'); put_u64(0ull - (uint64_t)v); } else put_u64((uint64_t)v);
  }
  __device__ __forceinline__ void put2(int v) { put((uint8_t)('0' + v / 10)); put((uint8_t)('0' + v % 10)); }
};

}  // namespace dxa
