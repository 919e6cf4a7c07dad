// Schema-driven synthetic JSON event generator for gfx950 (kernel K24) — the MI355X-side
// SimulatedData source (reference generators: Services/DataX.SimulatedData/DataX.SimulatedData.DataGenService/
// DataGen.cs:54-227 and DataProcessing/datax-utility/src/main/scala/datax/utility/DataGenerator.scala:27-167).
//
// A host compiler turns a schema into a tiny op program + literal pool; one lane renders one event.  Two passes:
// lengths (no stores) → exclusive scan on the stream → render into the final buffer, so events are packed
// back-to-back with exact offsets, ready for the JSON parser.  Randomness is counter-based (fmix64 of
// seed/event/op), hence deterministic and identical to the host reference implementation.
#include "dxa_common.h"
#include "dxa_emit.h"

namespace {

enum : int32_t {
  OP_LIT = 0,        // a: pool offset, b: length
  OP_INT = 1,        // a,b: [min, max) as int64 via (a | b<<32) pairs in ext
  OP_DBL = 2,        // ext: min(double), max(double); a: decimals
  OP_CHOICE = 3,     // a: table start (entries of (off,len) in table array), b: count
  OP_TS_MS = 4,      // epoch millis = base_ms + row * step_us / 1000
  OP_TS_STR = 5,     // a: format (0 "MM/dd/yyyy HH:mm:ss", 1 "yyyy-MM-ddTHH:mm:ssZ", 2 "yyyy-MM-dd HH:mm:ss")
  OP_BOOL = 6,
  OP_ALNUM = 7,      // a: length
  OP_NULLP = 8,      // a: probability per mille of emitting `null` instead of the next b ops
};

struct Op {
  int32_t code, a, b, pad;
  int64_t x, y;      // int range / double bits
};

struct GenArgs {
  const Op* ops;
  int32_t nops;
  const uint8_t* pool;
  const int32_t* table;   // (off,len) pairs for OP_CHOICE
  int32_t pool_words;     // pool size in 8-B words (padded)
  int32_t table_ints;     // table size in int32s
  uint64_t seed;
  int64_t row0;           // global index of the first event (for multi-batch determinism)
  int64_t n;
  int64_t base_ms;
  int64_t step_us;
  const int64_t* offs;    // write pass: [n+1]
  uint8_t* out;           // write pass
  int64_t* lens;          // length pass
  int64_t stride;         // slotted pass: bytes per event slot (16-B multiple, >= the program's length bound)
  int64_t* ends;          // slotted pass: [n] record ends (offs [n+1] are the slot starts)
};

__device__ __forceinline__ uint64_t rnd(uint64_t seed, int64_t row, int k) {
  return dxa::fmix64(seed ^ dxa::fmix64((uint64_t)row * dxa::kGold + (uint64_t)k * 0x632BE59BD9B4E019ull));
}

// A value in [0, span) from 64 random bits: multiply-shift of the top 32 bits for spans below 2^32 (no 64-bit
// software division per field; datagen.py _pick is the host twin), the remainder above.
__device__ __forceinline__ uint64_t pick(uint64_t r, uint64_t span) {
  return span <= 0xffffffffull ? ((r >> 32) * span) >> 32 : r % span;
}

__device__ __forceinline__ void civil(int64_t days, int64_t& y, int& m, int& d) {
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const unsigned doe = (unsigned)(days - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = (int64_t)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = (int)(doy - (153 * mp + 2) / 5 + 1);
  m = (int)(mp < 10 ? mp + 3 : mp - 9);
  if (m <= 2) ++y;
}

// little-endian text constants for put_word
constexpr uint64_t kTrue = 0x65757274ull;          // "true"
constexpr uint64_t kFalse = 0x65736c6166ull;       // "false"
constexpr uint64_t kNull = 0x6c6c756eull;          // "null"

// The program tables (ops, literal pool, choice table) as the render loop reads them: staged in LDS by the kernels
// (uniform reads broadcast from LDS; from global memory the compiler must assume the output stores may alias them
// and re-issues every read as a vector load).
struct Tables {
  const Op* ops;
  const uint64_t* pool64;   // literal runs and choice strings start 8-B aligned and are zero-padded (datagen.py)
  const int32_t* table;
};

template <bool WRITE>
__device__ __forceinline__ int64_t render(const GenArgs& g, const Tables& t, int64_t i, uint8_t* dst) {
  dxa::Emitter<WRITE> e(dst);
  const uint64_t* pool64 = t.pool64;
  const int64_t row = g.row0 + i;
  int skip = 0;
  for (int k = 0; k < g.nops; ++k) {
    const Op op = t.ops[k];
    if (skip > 0) { --skip; continue; }
    switch (op.code) {
      case OP_LIT:
        e.put_text_words(pool64 + (op.a >> 3), op.b);
        break;
      case OP_INT: {
        const uint64_t span = (uint64_t)(op.y - op.x);
        const int64_t v = op.x + (int64_t)(span ? pick(rnd(g.seed, row, k), span) : 0);
        e.put_i64(v);
        break;
      }
      case OP_DBL: {
        const double lo = __longlong_as_double(op.x), hi = __longlong_as_double(op.y);
        const double u = (double)(rnd(g.seed, row, k) >> 11) * (1.0 / 9007199254740992.0);
        const double v = lo + u * (hi - lo);
        uint64_t scale = 1;
        for (int q = 0; q < op.a; ++q) scale *= 10;
        const int64_t fixed = (int64_t)llround(v * (double)scale);
        const bool neg = fixed < 0;
        const uint64_t af = neg ? (0ull - (uint64_t)fixed) : (uint64_t)fixed;
        if (neg) e.put('-');
        // af / scale without a 64-bit software division: a double estimate, corrected by one step either way
        uint64_t ip;
        if (af < (1ull << 52)) {
          ip = (uint64_t)((double)af / (double)scale);
          if (ip * scale > af) --ip;
          if ((ip + 1) * scale <= af) ++ip;
        } else {
          ip = af / scale;
        }
        e.put_u64(ip);
        if (op.a > 0) {
          e.put('.');
          const uint64_t frac = af - ip * scale;
          if (op.a <= 8) {
            e.put_fixed((uint32_t)frac, (uint32_t)op.a);
          } else {
            uint64_t div = scale / 10;
            for (int q = 0; q < op.a; ++q) { e.put((uint8_t)('0' + (frac / div) % 10)); div = div > 1 ? div / 10 : 1; }
          }
        }
        break;
      }
      case OP_CHOICE: {
        const int idx = (int)pick(rnd(g.seed, row, k), (uint64_t)op.b);
        const int off = t.table[2 * (op.a + idx)], len = t.table[2 * (op.a + idx) + 1];
        e.put_text_words(pool64 + (off >> 3), len);
        break;
      }
      case OP_TS_MS:
        e.put_i64(g.base_ms + (row * g.step_us) / 1000 + op.x);
        break;
      case OP_TS_STR: {
        const int64_t secs = (g.base_ms + (row * g.step_us) / 1000) / 1000 + op.x;
        int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
        int64_t sod = secs - days * 86400;
        int64_t y; int m, d;
        civil(days, y, m, d);
        const int hh = (int)(sod / 3600), mi = (int)(sod / 60 % 60), ss = (int)(sod % 60);
        e.put('"');
        if (op.a == 0) {
          e.put2(m); e.put('/'); e.put2(d); e.put('/'); e.put_i64(y); e.put(' ');
        } else {
          if (y >= 1000 && y <= 9999) e.put_fixed((uint32_t)y, 4); else e.put_i64(y);
          e.put('-'); e.put2(m); e.put('-'); e.put2(d); e.put(op.a == 1 ? 'T' : ' ');
        }
        e.put2(hh); e.put(':'); e.put2(mi); e.put(':'); e.put2(ss);
        if (op.a == 1) e.put('Z');
        e.put('"');
        break;
      }
      case OP_BOOL:
        if (rnd(g.seed, row, k) & 1) e.put_word(kTrue, 4);
        else e.put_word(kFalse, 5);
        break;
      case OP_ALNUM: {
        e.put('"');
        uint64_t r = rnd(g.seed, row, k);
        uint64_t w = 0;
        uint32_t nw = 0;
        for (int q = 0; q < op.a; ++q) {
          if ((q & 7) == 7) r = dxa::fmix64(r + q);
          const int c = (int)(r % 62);
          r /= 62;
          w |= (uint64_t)(c < 10 ? '0' + c : (c < 36 ? 'A' + c - 10 : 'a' + c - 36)) << (8 * nw);
          if (++nw == 8) { e.put_word(w, 8); w = 0; nw = 0; }
        }
        if (nw) e.put_word(w, nw);
        e.put('"');
        break;
      }
      case OP_NULLP:
        if ((int)(rnd(g.seed, row, k) % 1000) < op.a) {
          e.put_word(kNull, 4);
          skip = op.b;
        }
        break;
      default:
        break;
    }
  }
  e.finish();
  return e.len;
}

__host__ __device__ __forceinline__ size_t lds_bytes_dev(int32_t nops, int32_t pool_words, int32_t table_ints) {
  return (size_t)nops * sizeof(Op) + (size_t)pool_words * 8 + (size_t)table_ints * 4;
}

// LDS image of the tables: ops (32 B each), pool words, table ints — sizes from the host (lds_bytes)
__device__ __forceinline__ Tables stage_tables(const GenArgs& g, uint64_t* smem) {
  const int op_words = g.nops * (int)(sizeof(Op) / 8);
  const uint64_t* src_ops = reinterpret_cast<const uint64_t*>(g.ops);
  const uint64_t* src_pool = reinterpret_cast<const uint64_t*>(g.pool);
  for (int q = threadIdx.x; q < op_words; q += blockDim.x) smem[q] = src_ops[q];
  uint64_t* pool = smem + op_words;
  for (int q = threadIdx.x; q < g.pool_words; q += blockDim.x) pool[q] = src_pool[q];
  int32_t* table = reinterpret_cast<int32_t*>(pool + g.pool_words);
  for (int q = threadIdx.x; q < g.table_ints; q += blockDim.x) table[q] = g.table[q];
  __syncthreads();
  return Tables{reinterpret_cast<const Op*>(smem), pool, table};
}

__global__ __launch_bounds__(256) void gen_len_kernel(GenArgs g) {
  extern __shared__ uint64_t smem[];
  const Tables t = stage_tables(g, smem);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  g.lens[i] = render<false>(g, t, i, nullptr);
}

__global__ __launch_bounds__(256) void gen_write_kernel(GenArgs g) {
  extern __shared__ uint64_t smem[];
  const Tables t = stage_tables(g, smem);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  render<true>(g, t, i, g.out + g.offs[i]);
}

// One pass, no length pass or scan: event i renders into its own 16-B aligned slot [i*stride, i*stride+len) (the
// host bounds every op's text, so len <= stride) and publishes its slot start and record end.  The parser takes
// (offs, ends) records with gaps as it does for Kafka values, so the batch needs no host read of its total size.
__global__ __launch_bounds__(256) void gen_slot_kernel(GenArgs g) {
  extern __shared__ uint64_t smem[];
  const Tables t = stage_tables(g, smem);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  const int64_t start = i * g.stride;
  const int64_t len = render<true>(g, t, i, g.out + start);
  const_cast<int64_t*>(g.offs)[i] = start;
  // len <= stride by construction (GenProgram.max_len bounds every op's text); were the bound ever wrong, the row
  // is published empty so the parser reports it malformed instead of reading into the next slot
  g.ends[i] = start + (len <= g.stride ? len : 0);
  if (i == g.n - 1) const_cast<int64_t*>(g.offs)[g.n] = g.n * g.stride;
}

size_t lds_bytes(int32_t nops, int32_t pool_words, int32_t table_ints) { return lds_bytes_dev(nops, pool_words, table_ints); }

constexpr size_t kMaxLds = 64 * 1024;

}  // namespace

DXA_API int dxa_datagen_op_size() { return (int)sizeof(Op); }

DXA_API int dxa_datagen_lengths(const void* ops, int32_t nops, const uint8_t* pool, int32_t pool_words,
                                const int32_t* table, int32_t table_ints, uint64_t seed, int64_t row0, int64_t n,
                                int64_t base_ms, int64_t step_us, int64_t* lens, void* st) {
  if (n <= 0) return 0;
  const size_t lds = lds_bytes(nops, pool_words, table_ints);
  if (lds > kMaxLds) return (int)hipErrorInvalidValue;
  GenArgs g{(const Op*)ops, nops, pool, table, pool_words, table_ints, seed, row0, n, base_ms, step_us, nullptr,
            nullptr, lens, 0, nullptr};
  hipLaunchKernelGGL(gen_len_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), lds, (hipStream_t)st, g);
  return (int)hipGetLastError();
}

DXA_API int dxa_datagen_write(const void* ops, int32_t nops, const uint8_t* pool, int32_t pool_words,
                              const int32_t* table, int32_t table_ints, uint64_t seed, int64_t row0, int64_t n,
                              int64_t base_ms, int64_t step_us, const int64_t* offs, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  const size_t lds = lds_bytes(nops, pool_words, table_ints);
  if (lds > kMaxLds) return (int)hipErrorInvalidValue;
  GenArgs g{(const Op*)ops, nops, pool, table, pool_words, table_ints, seed, row0, n, base_ms, step_us, offs, out,
            nullptr, 0, nullptr};
  hipLaunchKernelGGL(gen_write_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256),
                     lds, (hipStream_t)st, g);
  return (int)hipGetLastError();
}

DXA_API int dxa_datagen_slotted(const void* ops, int32_t nops, const uint8_t* pool, int32_t pool_words,
                                const int32_t* table, int32_t table_ints, uint64_t seed, int64_t row0, int64_t n,
                                int64_t base_ms, int64_t step_us, int64_t stride, int64_t* offs, int64_t* ends,
                                uint8_t* out, void* st) {
  if (n <= 0) return 0;
  if (stride <= 0 || (stride & 15)) return (int)hipErrorInvalidValue;
  const size_t lds = lds_bytes(nops, pool_words, table_ints);
  if (lds > kMaxLds) return (int)hipErrorInvalidValue;
  GenArgs g{(const Op*)ops, nops, pool, table, pool_words, table_ints, seed, row0, n, base_ms, step_us, offs, out,
            nullptr, stride, ends};
  hipLaunchKernelGGL(gen_slot_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), lds, (hipStream_t)st, g);
  return (int)hipGetLastError();
}
