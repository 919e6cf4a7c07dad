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
