// Kafka record framing on the GPU (record-batch v2, after the LZ4 decode of its records section).
//
// The host (host_kafka.cpp: dxa_kafka_plan) walks only the batch headers of a Fetch response and gives each batch
// its record count, the first record to keep and where its decompressed records start (its first LZ4 block's
// output slot).  This kernel walks each batch's records — one lane per batch, records are a serial chain of
// zig-zag varint headers — and writes every kept record's value range: [starts[i], ends[i]) in the decompressed
// buffer, in Kafka offset order across batches.  The JSON parser then reads the values in place (no copy).
// (kafka_frame_compact_kernel first closes the gaps of frames whose blocks are smaller than their slots.)
//
// Record: length varint | attributes i8 | timestampDelta varlong | offsetDelta varint | keyLength varint | key |
//         valueLength varint | value | headerCount varint | headers…
// Header bytes are read through a 32-byte register window (two aligned 16-B loads), so a record costs one or two
// dependent loads, not one per varint byte.  A batch whose blocks did not decode or whose records do not fill
// exactly its bytes gets empty values (parsed as malformed rows) and a nonzero bstatus, which the caller checks
// after the batch.
#include "dxa_common.h"

namespace {

struct Win {
  const uint8_t* base;
  int64_t wb;                  // window start (16-B aligned address offset from base), -1: empty
  uint4 a, b;
  __device__ __forceinline__ uint32_t at(int64_t q) {
    const uintptr_t addr = reinterpret_cast<uintptr_t>(base + q);
    const int64_t aq = q - (int64_t)(addr & 15);
    if (q - wb >= 32 || q < wb) {
      wb = aq;
      const uint4* w = reinterpret_cast<const uint4*>(base + aq);
      a = w[0];
      b = w[1];
    }
    const uint32_t o = (uint32_t)(q - wb);
    return o < 16 ? dxa::window_byte(a, o) : dxa::window_byte(b, o - 16);
  }
};

// zig-zag varint (up to 10 bytes); false on overrun
__device__ __forceinline__ bool varint(Win& w, int64_t& p, int64_t end, int64_t& v) {
  uint64_t u = 0;
  for (int s = 0; s < 70; s += 7) {
    if (p >= end) return false;
    const uint32_t c = w.at(p++);
    u |= (uint64_t)(c & 0x7f) << s;
    if (!(c & 0x80)) {
      v = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
      return true;
    }
  }
  return false;
}

// Frames whose non-final blocks are shorter than their slot (a producer block size below the frame's declared
// maximum) are made contiguous: one wave per batch moves its blocks down, in order, 16 bytes per lane (a block's
// destination never overlaps a later block's source, and blocks move in ascending order, so earlier moves only
// overwrite bytes already moved).  Contiguous frames — Kafka's 64 KiB blocks, single-block batches — exit at once.
__global__ __launch_bounds__(256) void kafka_frame_compact_kernel(uint8_t* __restrict__ buf, int64_t nbat,
                                                                  const int32_t* __restrict__ b_first,
                                                                  const int32_t* __restrict__ b_nblk,
                                                                  const int64_t* __restrict__ k_out_off,
                                                                  const int64_t* __restrict__ k_cap,
                                                                  const int64_t* __restrict__ produced,
                                                                  const int32_t* __restrict__ blk_status) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= nbat) return;
  const int32_t first = b_first[i], nb = b_nblk[i];
  bool gap = false;
  for (int32_t k = 0; k + 1 < nb; ++k) gap |= produced[first + k] != k_cap[first + k] || blk_status[first + k] != 0;
  if (!gap) return;
  int64_t dst = k_out_off[first] + produced[first];
  for (int32_t k = 1; k < nb; ++k) {
    const int64_t src = k_out_off[first + k], len = blk_status[first + k] != 0 ? 0 : produced[first + k];
    for (int64_t base = 0; base < len; base += 64) {              // ascending bytewise: dst <= src (memmove-safe)
      const int64_t q = base + lane;
      uint8_t v = 0;
      if (q < len) v = buf[src + q];
      __builtin_amdgcn_s_waitcnt(0);                            // every lane's load precedes any lane's store
      __builtin_amdgcn_wave_barrier();
      if (q < len) buf[dst + q] = v;
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
    }
    dst += len;
  }
}

__global__ __launch_bounds__(256) void kafka_records_kernel(
    const uint8_t* __restrict__ buf, int64_t nbat, const int32_t* __restrict__ b_count,
    const int32_t* __restrict__ b_skip, const int32_t* __restrict__ b_keep, const int32_t* __restrict__ b_first,
    const int32_t* __restrict__ b_nblk,
    const int64_t* __restrict__ b_rec0, const int64_t* __restrict__ k_out_off, const int64_t* __restrict__ k_cap,
    const int64_t* __restrict__ produced, const int32_t* __restrict__ blk_status, int64_t* __restrict__ starts,
    int64_t* __restrict__ ends, int32_t* __restrict__ bstatus) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nbat) return;
  // records [skip, skip + keep) are emitted (keep < count - skip: a rate limit cut the batch)
  const int32_t count = b_count[i], skip = b_skip[i], first = b_first[i], nb = b_nblk[i];
  const int32_t stop = skip + b_keep[i] < count ? skip + b_keep[i] : count;
  const int64_t r0 = b_rec0[i];
  int32_t rc = 0;
  int64_t total = 0;                                              // frame bytes (contiguous after the compaction)
  for (int32_t k = 0; k < nb; ++k) {
    if (blk_status[first + k] != 0) rc = 1;                       // block did not decode
    total += produced[first + k];
  }
  int64_t p = k_out_off[first];
  const int64_t end = p + (rc == 1 ? 0 : total);
  Win w{buf, -64, make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  int32_t r = 0;
  for (; rc == 0 && r < stop; ++r) {
    int64_t len, tsd, od, klen, vlen;
    if (!varint(w, p, end, len) || len < 0 || p + len > end) { rc = 3; break; }
    const int64_t rec_end = p + len;
    ++p;                                                          // attributes
    if (!varint(w, p, rec_end, tsd) || !varint(w, p, rec_end, od) || !varint(w, p, rec_end, klen)) {
      rc = 4;
      break;
    }
    if (klen > 0) p += klen;
    if (!varint(w, p, rec_end, vlen) || p + (vlen > 0 ? vlen : 0) > rec_end) { rc = 5; break; }
    if (r >= skip) {
      const int64_t o = r0 + (r - skip);
      starts[o] = p;
      ends[o] = p + (vlen > 0 ? vlen : 0);                       // null value: empty record
    }
    p = rec_end;
  }
  if (rc == 0 && stop == count && p != end) rc = 6;                // records must fill the batch's bytes exactly
  if (rc != 0) {
    for (int32_t q = (r > skip ? r : skip); q < stop; ++q) {     // the rest of the batch: empty values
      starts[r0 + (q - skip)] = 0;
      ends[r0 + (q - skip)] = 0;
    }
  }
  bstatus[i] = rc;
}


// ---- CRC-32C of every record batch, on the device (the consumer's check.crcs) -------------------------------------
// The CRC covers a batch from its attributes field to its end (~16 KiB for a 16 KiB producer batch), over the
// compressed bytes already in HBM, so the host planner touches no record bytes (a host CRC would read every fetched
// byte once more from host memory — ~55 GB/s per GPU at the groupby rate, on top of the DMA's own reads).
//
// One wave per batch, lane-interleaved: the bytes are cut into 512-B rows right-aligned on the 8-B boundary at or
// below the batch end, and lane l owns the 8-B word at l*8 of every row — one coalesced 512-B load per row.  The
// zero-init ("raw") CRC register is linear in the message, so each lane accumulates its words as if every other
// byte were zero: acc = T8(acc ^ w) (slice-by-8: "process 8 bytes") then acc = acc·x^(8·504) (the 504 zero bytes
// of the other lanes, a 4-table constant multiply).  After the last row lane l is still (63-l)·8 bytes from the
// end: acc·x^(64·(63-l)) (per-lane constant, precomputed), XOR-reduced over the wave.  The 0xFFFFFFFF init is
// folded into the message (XOR into its first 4 bytes); bytes before the batch start load as zero (no effect on a
// zero-init register); lane 0 finishes the < 8-B tail serially and inverts.  LDS holds only the tables (12 KiB), so
// the check shares CUs with the LZ4 decode it runs beside (side stream).  Writes 7 (mismatch) or 0 per batch.
constexpr uint32_t kCrcPoly = 0x82F63B78u;

__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 1
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

// x^(8n) mod P (reflected) by square-and-multiply from x^1
__device__ uint32_t x8n(uint64_t n) {
  uint32_t p = 1u << 31, sq = 1u << 30;         // x^0, x^1
  for (int q = 0; q < 3; ++q) sq = multmodp(sq, sq);
  for (; n; n >>= 1) {
    if (n & 1) p = multmodp(sq, p);
    sq = multmodp(sq, sq);
  }
  return p;
}

__global__ __launch_bounds__(256) void kafka_crc_kernel(const uint8_t* __restrict__ data, int64_t nbat,
                                                        const int64_t* __restrict__ b_off,
                                                        const int32_t* __restrict__ b_len,
                                                        const int32_t* __restrict__ b_want,
                                                        int32_t* __restrict__ bstatus) {
  __shared__ uint32_t t8[8][256];          // slice-by-8
  __shared__ uint32_t m504[4][256];        // multiply by x^(8*504)
  const int tid = threadIdx.x, lane = tid & 63;
  {
    uint32_t c = (uint32_t)tid;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    t8[0][tid] = c;
    const uint32_t k504 = x8n(504);
    for (int j = 0; j < 4; ++j) m504[j][tid] = multmodp(k504, (uint32_t)tid << (8 * j));
    for (int t = 1; t < 8; ++t) {
      __syncthreads();
      t8[t][tid] = (t8[t - 1][tid] >> 8) ^ t8[0][t8[t - 1][tid] & 0xff];
    }
    __syncthreads();
  }
  const uint32_t kend = x8n((uint64_t)(63 - lane) * 8);   // this lane's distance to the end of a row
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (tid >> 6); i < nbat; i += waves) {
    const int64_t s = b_off[i], e = s + b_len[i];
    int64_t E = e - (int64_t)(reinterpret_cast<uintptr_t>(data + e) & 7);          // 8-B aligned end
    if (E - s < 8) E = s;                                      // tiny batch: all serial (init not folded)
    const int64_t nrow = (E - s + 511) / 512;
    const int64_t r0 = E - nrow * 512;                         // 8-B aligned; row 0 may start before s
    uint32_t acc = 0;
    for (int64_t r = 0; r < nrow; ++r) {
      const int64_t a = r0 + r * 512 + lane * 8;
      uint64_t w = 0;
      if (a + 8 > s) {
        w = *reinterpret_cast<const uint64_t*>(data + a);
        if (a < s + 4) {                                       // zero bytes before s, XOR the init into s..s+3
          const int64_t lo = s - a;                            // may be negative
          const uint64_t keep = lo > 0 ? (~0ull << (8 * lo)) : ~0ull;
          const int64_t x0 = lo > 0 ? lo : 0, x1 = lo + 4 < 8 ? lo + 4 : 8;
          uint64_t inv = 0;
          for (int64_t q = x0; q < x1; ++q) inv |= 0xffull << (8 * q);
          w = (w & keep) ^ inv;
        }
      }
      acc = (uint32_t)(acc ^ (uint32_t)w);
      const uint32_t hi = (uint32_t)(w >> 32);
      acc = t8[7][acc & 0xff] ^ t8[6][(acc >> 8) & 0xff] ^ t8[5][(acc >> 16) & 0xff] ^ t8[4][acc >> 24] ^
            t8[3][hi & 0xff] ^ t8[2][(hi >> 8) & 0xff] ^ t8[1][(hi >> 16) & 0xff] ^ t8[0][hi >> 24];
      if (r + 1 < nrow)
        acc = m504[0][acc & 0xff] ^ m504[1][(acc >> 8) & 0xff] ^ m504[2][(acc >> 16) & 0xff] ^ m504[3][acc >> 24];
    }
    uint32_t term = acc ? multmodp(kend, acc) : 0u;
    for (int off = 32; off; off >>= 1) term ^= (uint32_t)__shfl_xor((int)term, off, 64);
    if (lane == 0) {
      uint32_t c = E > s ? term : 0xFFFFFFFFu;                 // raw register after [s, E); continue the tail
      for (int64_t p = E; p < e; ++p) c = (c >> 8) ^ t8[0][(c ^ data[p]) & 0xff];
      bstatus[i] = ~c != (uint32_t)b_want[i] ? 7 : 0;
    }
  }
}

}  // namespace

DXA_API int dxa_kafka_records(const uint8_t* buf, int64_t nbat, const int32_t* b_count, const int32_t* b_skip,
                              const int32_t* b_keep, const int32_t* b_first, const int32_t* b_nblk,
                              const int64_t* b_rec0,
                              const int64_t* k_out_off, const int64_t* k_cap, const int64_t* produced,
                              const int32_t* blk_status, int64_t* starts, int64_t* ends, int32_t* bstatus,
                              void* stream) {
  if (nbat <= 0) return 0;
  hipLaunchKernelGGL(kafka_frame_compact_kernel, dim3((unsigned)((nbat * 64 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, const_cast<uint8_t*>(buf), nbat, b_first, b_nblk, k_out_off, k_cap,
                     produced, blk_status);
  hipLaunchKernelGGL(kafka_records_kernel, dim3((unsigned)((nbat + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     buf, nbat, b_count, b_skip, b_keep, b_first, b_nblk, b_rec0, k_out_off, k_cap, produced,
                     blk_status, starts, ends, bstatus);
  return (int)hipGetLastError();
}

// Verify every planned batch's CRC-32C: cstatus[i] = 7 on a mismatch, 0 otherwise.
DXA_API int dxa_kafka_crc(const uint8_t* data, int64_t nbat, const int64_t* b_off, const int32_t* b_len,
                          const int32_t* b_want, int32_t* bstatus, void* stream) {
  if (nbat <= 0) return 0;
  // grid-strided over the batches, 4 waves (one batch each) per workgroup; tables built once per workgroup
  const int64_t blocks = (nbat + 3) / 4;
  hipLaunchKernelGGL(kafka_crc_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0,
                     (hipStream_t)stream, data, nbat, b_off, b_len, b_want, bstatus);
  return (int)hipGetLastError();
}
