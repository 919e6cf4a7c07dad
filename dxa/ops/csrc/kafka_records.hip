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
// The CRC covers a batch from its attributes field to its end (~16 KiB for a 16 KiB producer batch), in the
// compressed bytes already in HBM, so the host planner touches no record bytes at all (host CRC would read every
// fetched byte once more from host memory — ~55 GB/s per GPU at the groupby rate, on top of the DMA's own reads).
// One wave per batch: lane l takes the contiguous segment [l*seg, (l+1)*seg) and runs slice-by-8 table CRC over it
// (tables in LDS); the 64 finalized segment CRCs are combined as crc(AB) = x^(8|B|)·crc(A) ⊕ crc(B) in GF(2)[x]/P
// (reflected, zlib's multmodp/x2nmodp with the Castagnoli polynomial), i.e. each lane scales its CRC by
// x^(8·bytes after its segment) and the wave XOR-reduces.  Writes 7 (mismatch) or 0 per batch into its own status
// array, so the check runs on a side stream concurrently with the LZ4 decode and record framing.
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

__global__ __launch_bounds__(256) void kafka_crc_kernel(const uint8_t* __restrict__ data, int64_t nbat,
                                                        const int64_t* __restrict__ b_off,
                                                        const int32_t* __restrict__ b_len,
                                                        const int32_t* __restrict__ b_want,
                                                        int32_t* __restrict__ bstatus) {
  __shared__ uint32_t tab[8][256];
  __shared__ uint32_t x2n[32];
  const int tid = threadIdx.x;
  {
    uint32_t c = (uint32_t)tid;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    tab[0][tid] = c;
    for (int t = 1; t < 8; ++t) {
      // tab[t][i] = (tab[t-1][i] >> 8) ^ tab[0][tab[t-1][i] & 0xff]: needs all of tab[0] first
      __syncthreads();
      tab[t][tid] = (tab[t - 1][tid] >> 8) ^ tab[0][tab[t - 1][tid] & 0xff];
    }
    if (tid < 32) {                                   // x^(2^k) mod P, reflected (x^1 = bit 30)
      uint32_t p = 1u << 30;
      for (int k = 0; k < tid; ++k) p = multmodp(p, p);
      x2n[tid] = p;
    }
    __syncthreads();
  }
  const int lane = tid & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (tid >> 6); i < nbat; i += waves) {
    const int64_t n = b_len[i];
    const uint8_t* base = data + b_off[i];
    const int64_t seg = (((n + 63) >> 6) + 7) & ~(int64_t)7;
    const int64_t lo = lane * seg < n ? lane * seg : n;
    const int64_t hi = lo + seg < n ? lo + seg : n;
    uint32_t c = 0xFFFFFFFFu;
    const uint8_t* q = base + lo;
    const uint8_t* e = base + hi;
    while (q < e && ((uintptr_t)q & 7)) c = (c >> 8) ^ tab[0][(c ^ *q++) & 0xff];
    for (; q + 8 <= e; q += 8) {
      const uint2 w = *reinterpret_cast<const uint2*>(q);
      const uint32_t lo32 = w.x ^ c, hi32 = w.y;
      c = tab[7][lo32 & 0xff] ^ tab[6][(lo32 >> 8) & 0xff] ^ tab[5][(lo32 >> 16) & 0xff] ^ tab[4][lo32 >> 24] ^
          tab[3][hi32 & 0xff] ^ tab[2][(hi32 >> 8) & 0xff] ^ tab[1][(hi32 >> 16) & 0xff] ^ tab[0][hi32 >> 24];
    }
    while (q < e) c = (c >> 8) ^ tab[0][(c ^ *q++) & 0xff];
    uint32_t crc = (hi > lo) ? ~c : 0u;               // CRC-32C of an empty segment is 0
    // scale by x^(8 * bytes after this segment)
    uint64_t after = (uint64_t)(n - hi);
    uint32_t sc = 1u << 31;                            // x^0
    for (int k = 3; after; after >>= 1, ++k)
      if (after & 1) sc = multmodp(x2n[k & 31], sc);
    uint32_t term = crc ? multmodp(sc, crc) : 0u;
    for (int off = 32; off; off >>= 1) term ^= (uint32_t)__shfl_xor((int)term, off, 64);
    if (lane == 0) bstatus[i] = term != (uint32_t)b_want[i] ? 7 : 0;
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
  const int64_t blocks = (nbat + 3) / 4;
  hipLaunchKernelGGL(kafka_crc_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0,
                     (hipStream_t)stream, data, nbat, b_off, b_len, b_want, bstatus);
  return (int)hipGetLastError();
}
