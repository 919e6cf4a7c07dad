// LZ4 block decoder for gfx950: compressed ingest (LZ4-frame event batches, Kafka compression codec 3) is
// decompressed in HBM after a compressed H2D copy, so PCIe carries ~2.5x fewer bytes per event.
//
// Decoder: 16 lanes per block, output straight to HBM (lz4_decode_group_kernel, design notes below).  A size pass
// (one lane per block, register-window input, no stores) serves frames whose blocks do not carry decompressed sizes.
// Measured and dropped (profiles/kafka_batching/README.md): one wave per block with LDS-staged output, one lane per
// block, 8 lanes per block.
#include "dxa_common.h"

namespace {

struct InWin {
  const uint8_t* base;
  uintptr_t wb;
  uint4 w;
  __device__ __forceinline__ uint32_t at(int64_t q) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(base + q);
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != wb) {
      wb = b;
      w = *reinterpret_cast<const uint4*>(b);
    }
    return dxa::window_byte(w, (uint32_t)(a - b));
  }
};

struct OutBuf {
  uint8_t* p;
  int64_t len;
  int head;                 // bytes written singly until p + len is 16-B aligned
  int nacc;
  uint64_t a0, a1;
  uintptr_t wb;             // read-back window over flushed output
  uint4 w;

  __device__ __forceinline__ void init(uint8_t* dst) {
    p = dst; len = 0; nacc = 0; a0 = a1 = 0; wb = 0;
    head = (int)((16 - ((uintptr_t)dst & 15)) & 15);
  }
  __device__ __forceinline__ void put(uint32_t c) {
    if (len < head) {
      p[len] = (uint8_t)c;
      wb = 0;                                   // a cached window may cover this byte
    } else {
      if (nacc < 8) a0 |= (uint64_t)c << (8 * nacc);
      else a1 |= (uint64_t)c << (8 * (nacc - 8));
      if (++nacc == 16) {
        uint64_t* q = reinterpret_cast<uint64_t*>(p + len - 15);
        __builtin_nontemporal_store(a0, q);
        __builtin_nontemporal_store(a1, q + 1);
        a0 = a1 = 0;
        nacc = 0;
      }
    }
    ++len;
  }
  // byte at output position q (< len)
  __device__ __forceinline__ uint32_t get(int64_t q) {
    const int64_t acc0 = len - nacc;
    if (q >= acc0 && len >= head) {
      const int k = (int)(q - acc0);
      return (uint32_t)(((k < 8) ? (a0 >> (8 * k)) : (a1 >> (8 * (k - 8)))) & 0xff);
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + q);
    const uintptr_t b = a & ~(uintptr_t)15;
    if (b != wb) {
      wb = b;
      asm volatile("" ::: "memory");            // keep the load after this lane's earlier stores (aliasing types)
      w = *reinterpret_cast<const uint4*>(b);
    }
    return dxa::window_byte(w, (uint32_t)(a - b));
  }
  __device__ __forceinline__ void finish() {
    uint8_t* q = p + len - nacc;
    for (int k = 0; k < nacc; ++k) q[k] = (uint8_t)((k < 8 ? a0 >> (8 * k) : a1 >> (8 * (k - 8))) & 0xff);
  }
};

enum : int32_t { LZ_OK = 0, LZ_TRUNC = 1, LZ_OFFSET = 2, LZ_OVERFLOW = 3, LZ_SIZE = 4 };

// Walk one block's sequences.  WRITE=false: count output bytes only.
template <bool WRITE>
__device__ int32_t run_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t& produced) {
  InWin in{src, 0, make_uint4(0, 0, 0, 0)};
  OutBuf out;
  if (WRITE) out.init(dst);
  int64_t ip = 0, op = 0;
  while (ip < n) {
    const uint32_t token = in.at(ip++);
    int64_t lit = token >> 4;
    if (lit == 15) {
      uint32_t b;
      do { if (ip >= n) return LZ_TRUNC; b = in.at(ip++); lit += b; } while (b == 255);
    }
    if (lit > n - ip) return LZ_TRUNC;
    if (lit > cap - op) return LZ_OVERFLOW;
    if (WRITE) for (int64_t k = 0; k < lit; ++k) out.put(in.at(ip + k));
    ip += lit;
    op += lit;
    if (ip >= n) break;
    if (n - ip < 2) return LZ_TRUNC;
    const int64_t off = (int64_t)in.at(ip) | ((int64_t)in.at(ip + 1) << 8);
    ip += 2;
    if (off == 0 || off > op) return LZ_OFFSET;
    int64_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do { if (ip >= n) return LZ_TRUNC; b = in.at(ip++); ml += b; } while (b == 255);
    }
    ml += 4;
    if (ml > cap - op) return LZ_OVERFLOW;
    if (WRITE) {
      const int64_t s = op - off;
      if (off == 1) {
        const uint32_t c = out.get(s);
        for (int64_t k = 0; k < ml; ++k) out.put(c);
      } else {
        for (int64_t k = 0; k < ml; ++k) out.put(out.get(s + k));
      }
    }
    op += ml;
  }
  if (WRITE) out.finish();
  produced = op;
  return LZ_OK;
}

__global__ __launch_bounds__(256) void lz4_sizes_kernel(const uint8_t* __restrict__ src,
                                                        const int64_t* __restrict__ comp_off,
                                                        const int32_t* __restrict__ comp_len,
                                                        const uint8_t* __restrict__ stored, int64_t nb,
                                                        int64_t max_block, int64_t* __restrict__ out_len,
                                                        int32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  if (stored[b]) { out_len[b] = comp_len[b]; status[b] = LZ_OK; return; }
  int64_t produced = 0;
  const int32_t rc = run_block<false>(src + comp_off[b], comp_len[b], nullptr, max_block, produced);
  out_len[b] = rc == LZ_OK ? produced : 0;
  status[b] = rc;
}

// ---- 16 lanes per block, output straight to HBM -----------------------------------------------------------
// Bench blocks have ~1400 sequences of ~1.7 literal + ~10 match bytes, so neither 64-wide copies nor a
// wave-uniform (scalar-unit) parser pays: the per-CU scalar unit serialises every wave's header chain.  Here a
// group of 16 lanes owns one block and keeps its sequence state in VGPRs, so one VALU instruction advances four
// blocks, and with no LDS per block every block of a batch can be resident at once (latency hidden by
// occupancy).
//   * Input window: lane k of the group holds dword k of a 64-byte window (one coalesced dword load per lane,
//     refilled every ~10 sequences); a byte at window offset r is ds_bpermute(lane r/4) >> 8*(r%4).
//   * Fast path (lit < 15, match code < 15, header + literals inside the window — nearly every JSON sequence):
//     straight-line code — token, per-lane literal byte and the 2 offset bytes from the window, then a
//     <= 18-byte match copy as two 16-lane steps.  Anything else takes the general path.
//   * Match sources precede op; a `s_waitcnt vmcnt(0)` before the copy makes earlier stores visible (a CU's
//     lanes share one L1, so a same-wave hand-off needs no cache maintenance).  Fast-path match bytes are stored
//     one sequence late (software pipelining), so their load latency overlaps the next header parse.  `done` tracks the output prefix
//     known complete at the last such wait, so the wait is only taken when a source reaches past it — about
//     once per `off` bytes (~600 B, one record) for JSON.
//   * The group width is a template parameter: G = 8 (eight blocks per instruction, a 2-dword window per lane,
//     4-byte-per-lane match copies) measured 6.07 ms against 4.72 ms for G = 16 on the bench batch.
//   * Measured and dropped (profiles/kafka_batching/README.md): an LDS history ring for match sources (the byte
//     stores to LDS and the occupancy it costs outweigh the HBM round trips it saves: 8.13 -> 8.71 / 12.61 ms per
//     groupby step with a 1 / 2 KiB ring) and branch-free masked stores (below).
constexpr int kWaitVm0 = 0xF70;                                        // s_waitcnt vmcnt(0) (gfx9 encoding)

template <int G>
__global__ __launch_bounds__(256) void lz4_decode_group_kernel(const uint8_t* __restrict__ src,
                                                               const int64_t* __restrict__ comp_off,
                                                               const int32_t* __restrict__ comp_len,
                                                               const uint8_t* __restrict__ stored,
                                                               const int64_t* __restrict__ out_off,
                                                               const int64_t* __restrict__ out_len, int64_t nb,
                                                               uint8_t* __restrict__ dst,
                                                               int32_t* __restrict__ status,
                                                               int64_t* __restrict__ produced) {
  // produced == null: out_len[b] is the exact decompressed size; else it is a capacity and the size is reported
  // in produced[b] (Kafka frames do not carry their content size)
  static_assert(G == 8 || G == 16, "group width");
  // 64-byte input window = NW dwords per lane; fast-path literals LPL bytes per lane; pipelined matches (<= 32 B)
  // BPL bytes per lane
  constexpr int NW = 16 / G, LPL = 16 / G, BPL = 32 / G, LOG_G = G == 8 ? 3 : 4;
  constexpr int WB = 64, PIPE = 32;
  const int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const int gl = (int)(threadIdx.x & (G - 1));
  const int gbase = (int)((threadIdx.x & 63) & ~(G - 1));
  if (b >= nb) return;
  const uint8_t kd = stored[b];            // 0 LZ4 block, 1 stored bytes, 2 deflate (inflate.hip's, skipped here)
  if (kd > 1) return;
  const int32_t n = comp_len[b];
  const int64_t cap64 = out_len[b];
  const uint8_t* in = src + comp_off[b];
  uint8_t* out = dst + out_off[b];
  // predicated byte stores / loads: the exec-mask branch around each skips the memory instruction when no lane of
  // the wave needs it (a branch-free variant storing masked-off lanes to a dump buffer measured 4.77 -> 5.84 ms on
  // 16 KiB blocks and 6.90 -> 8.48 ms on 64 KiB blocks: the extra stores cost more than the branches)
  auto put = [&](bool on, int32_t pos, uint32_t v) {
    if (on) out[pos] = (uint8_t)v;
  };
  auto fetch = [&](bool on, int32_t pos) -> uint32_t { return on ? (uint32_t)out[pos] : 0u; };
  if (kd) {
    if (produced ? (n > cap64) : (n != cap64)) {
      if (gl == 0) status[b] = LZ_SIZE;
      return;
    }
    for (int32_t k = gl; k < n; k += G) out[k] = in[k];
    if (gl == 0) {
      status[b] = LZ_OK;
      if (produced) produced[b] = n;
    }
    return;
  }
  if (cap64 > INT32_MAX || cap64 < 0 || n < 0) {
    if (gl == 0) status[b] = LZ_OVERFLOW;
    return;
  }
  const int32_t cap = (int32_t)cap64;
  const int32_t shift = (int32_t)(reinterpret_cast<uintptr_t>(in) & 3);
  const uint8_t* a0 = in - shift;
  const int32_t lim = shift + n + 16;
  uint32_t X[NW];
  auto ld = [&](int32_t w0) {
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int32_t q = w0 + 4 * (gl + G * k);
      X[k] = (q + 4 <= lim) ? *reinterpret_cast<const uint32_t*>(a0 + q) : 0u;
    }
    // wait here, inside the (rare) refill branch, with a wait the compiler can see: otherwise it waits for the
    // window register where the refill and no-refill paths merge, every sequence (vmcnt retires in order, so that
    // also drains the pipelined match loads).  Measured neutral on the bench batch (4.72 vs 4.74 ms): the header
    // chain, not that wait, sets the pace.
    __builtin_amdgcn_s_waitcnt(kWaitVm0);
  };
  auto wbyte = [&](int32_t r) -> uint32_t {
    const int d = (r >> 2) & (G * NW - 1);
    const int addr = (gbase + (d & (G - 1))) << 2;
    uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)X[0]);
    if constexpr (NW == 2) {
      const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)X[1]);
      v = (d >> LOG_G) ? v1 : v;
    }
    return (v >> ((r & 3) * 8)) & 0xffu;
  };
  int32_t xb = 0;
  ld(0);
  auto get = [&](int32_t p) -> uint32_t {
    if (p - xb >= WB) {
      xb = p & ~3;
      ld(xb);
    }
    return wbyte(p - xb);
  };
  const int32_t iend = shift + n;
  int32_t ip = shift, op = 0, rc = LZ_OK, done = 0;
  int32_t pdst = 0, pml = 0;
  uint32_t pv[BPL];
#pragma unroll
  for (int k = 0; k < BPL; ++k) pv[k] = 0;
  auto flush = [&]() {
#pragma unroll
    for (int k = 0; k < BPL; ++k) put(gl + G * k < pml, pdst + G * k + gl, pv[k]);
  };
  while (ip < iend) {
    if (ip - xb > WB - 16) {
      xb = ip & ~3;
      ld(xb);
    }
    const int32_t r = ip - xb;
    const uint32_t token = wbyte(r);
    int32_t lit = (int32_t)(token >> 4);
    const int32_t mlc = (int32_t)(token & 15);
    const bool has_ext = mlc == 15 && lit < 15 && r + lit + 4 <= WB;
    const uint32_t mext = has_ext ? wbyte(r + lit + 3) : 0u;
    const int32_t fml = mlc + 4 + (int32_t)mext;
    const int32_t fhdr = lit + 3 + (mlc == 15 ? 1 : 0);
    if (lit < 15 && (mlc < 15 || mext < 255) && r + fhdr <= WB && iend - ip >= fhdr && cap - op >= lit + fml) {
#pragma unroll
      for (int k = 0; k < LPL; ++k) {
        const uint32_t lv = wbyte(r + 1 + G * k + gl);
        put(gl + G * k < lit, op + G * k + gl, lv);
      }
      const int32_t off = (int32_t)(wbyte(r + 1 + lit) | (wbyte(r + 2 + lit) << 8));
      ip += fhdr;
      op += lit;
      if (off == 0 || off > op) { rc = LZ_OFFSET; break; }
      const int32_t ml = fml;
      const int32_t s0 = op - off;
      const int32_t src_end = s0 + (off < ml ? off : ml);
      if (pml > 0 && (src_end > pdst || ml > PIPE)) {
        flush();
        pml = 0;
      }
      if (src_end > done) {
        __builtin_amdgcn_s_waitcnt(kWaitVm0);
        asm volatile("" ::: "memory");
        done = pml > 0 ? pdst : op;
      }
      if (ml > PIPE) {
        if (off >= ml) {
          for (int32_t c = 0; c < ml; c += G)
            if (c + gl < ml) out[op + c + gl] = out[s0 + c + gl];
        } else {
          for (int32_t c = 0; c < ml; c += G) {
            const uint32_t i = (uint32_t)(c + gl);
            if ((int32_t)i < ml) out[op + i] = out[s0 + (int32_t)(i % (uint32_t)off)];
          }
        }
        op += ml;
        continue;
      }
      uint32_t v[BPL];
      if (off >= ml) {
#pragma unroll
        for (int k = 0; k < BPL; ++k) v[k] = fetch(gl + G * k < ml, s0 + G * k + gl);
      } else {
        const uint32_t o = (uint32_t)off;
#pragma unroll
        for (int k = 0; k < BPL; ++k) v[k] = fetch(gl + G * k < ml, s0 + (int32_t)((uint32_t)(gl + G * k) % o));
      }
      if (pml > 0) flush();
      pdst = op;
      pml = ml;
#pragma unroll
      for (int k = 0; k < BPL; ++k) pv[k] = v[k];
      op += ml;
      continue;
    }
    if (pml > 0) {
      flush();
      pml = 0;
    }
    ++ip;
    if (lit == 15) {
      uint32_t e;
      do {
        if (ip >= iend) { rc = LZ_TRUNC; break; }
        e = get(ip);
        ++ip;
        lit += (int32_t)e;
      } while (e == 255);
      if (rc != LZ_OK) break;
    }
    if (lit > iend - ip) { rc = LZ_TRUNC; break; }
    if (lit > cap - op) { rc = LZ_OVERFLOW; break; }
    for (int32_t c = 0; c < lit; c += G)
      if (c + gl < lit) out[op + c + gl] = a0[ip + c + gl];
    ip += lit;
    op += lit;
    if (ip >= iend) break;
    if (iend - ip < 2) { rc = LZ_TRUNC; break; }
    const int32_t off = (int32_t)(get(ip) | (get(ip + 1) << 8));
    ip += 2;
    if (off == 0 || off > op) { rc = LZ_OFFSET; break; }
    int32_t ml = mlc;
    if (ml == 15) {
      uint32_t e;
      do {
        if (ip >= iend) { rc = LZ_TRUNC; break; }
        e = get(ip);
        ++ip;
        ml += (int32_t)e;
      } while (e == 255);
      if (rc != LZ_OK) break;
    }
    ml += 4;
    if (ml > cap - op) { rc = LZ_OVERFLOW; break; }
    const int32_t s0 = op - off;
    if (s0 + (off < ml ? off : ml) > done) {
      __builtin_amdgcn_s_waitcnt(kWaitVm0);
      asm volatile("" ::: "memory");
      done = op;
    }
    if (off >= ml) {
      for (int32_t c = 0; c < ml; c += G)
        if (c + gl < ml) out[op + c + gl] = out[s0 + c + gl];
    } else {
      for (int32_t c = 0; c < ml; c += G) {
        const uint32_t i = (uint32_t)(c + gl);
        if ((int32_t)i < ml) out[op + i] = out[s0 + (int32_t)(i % (uint32_t)off)];
      }
    }
    op += ml;
  }
  if (pml > 0) flush();
  if (rc == LZ_OK && !produced && op != cap) rc = LZ_SIZE;
  if (gl == 0) {
    status[b] = rc;
    if (produced) produced[b] = op;
  }
}

}  // namespace

DXA_API int dxa_lz4_block_sizes(const void* src, const void* comp_off, const void* comp_len, const void* stored,
                                int64_t nb, int64_t max_block, void* out_len, void* status, void* st) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(lz4_sizes_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, (hipStream_t)st,
                     (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len, (const uint8_t*)stored,
                     nb, max_block, (int64_t*)out_len, (int32_t*)status);
  return (int)hipGetLastError();
}

// launch the G-lane group decoder (one block per G lanes)
template <int G>
static int launch_group(int64_t nb, hipStream_t s, const uint8_t* src, const int64_t* co, const int32_t* cl,
                        const uint8_t* sd, const int64_t* oo, const int64_t* ol, uint8_t* dst, int32_t* status,
                        int64_t* produced) {
  const dim3 grid((unsigned)((nb * G + 255) / 256));
  hipLaunchKernelGGL((lz4_decode_group_kernel<G>), grid, dim3(256), 0, s, src, co, cl, sd, oo, ol, nb, dst, status,
                     produced);
  return (int)hipGetLastError();
}

DXA_API int dxa_lz4_decode(const void* src, const void* comp_off, const void* comp_len, const void* stored,
                           const void* out_off, const void* out_len, int64_t nb, int64_t max_out, void* dst,
                           void* status, void* st) {
  if (nb <= 0) return 0;
  const hipStream_t s = (hipStream_t)st;
  return launch_group<16>(nb, s, (const uint8_t*)src, (const int64_t*)comp_off, (const int32_t*)comp_len,
                          (const uint8_t*)stored, (const int64_t*)out_off, (const int64_t*)out_len, (uint8_t*)dst,
                          (int32_t*)status, (int64_t*)nullptr);
}

// Blocks with a capacity instead of a known size (Kafka LZ4 frames): `cap[b]` bytes reserved at out_off[b], the
// decompressed size comes back in produced[b].  The group decoder, 16 lanes per block.
DXA_API int dxa_lz4_decode_into(const void* src, const void* comp_off, const void* comp_len, const void* stored,
                                const void* out_off, const void* cap, int64_t nb, void* dst, void* produced,
                                void* status, void* st) {
  if (nb <= 0) return 0;
  const hipStream_t s = (hipStream_t)st;
  const uint8_t* s8 = (const uint8_t*)src;
  const int64_t* co = (const int64_t*)comp_off;
  const int32_t* cl = (const int32_t*)comp_len;
  const uint8_t* sd = (const uint8_t*)stored;
  const int64_t* oo = (const int64_t*)out_off;
  const int64_t* cp = (const int64_t*)cap;
  return launch_group<16>(nb, s, s8, co, cl, sd, oo, cp, (uint8_t*)dst, (int32_t*)status, (int64_t*)produced);
}

// Async H2D copy of a byte range of a pinned host buffer on `st` (torch's copy_ of a pinned *slice* falls back
// to a host-synchronous copy, which would serialise the chunked ingest pipeline behind the host thread).
DXA_API int dxa_memcpy_h2d_async(void* dst, const void* src, int64_t n, void* st) {
  if (n <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyHostToDevice, (hipStream_t)st);
}
