// Device JSON-lines serializer (kernel K20): rows of a columnar table → newline-terminated JSON with
// Spark ``to_json(struct(*))`` semantics — field order = column order, null fields omitted, MAP nulls written as
// null, filterNull arrays skip nulls, timestamps as "yyyy-MM-dd'T'HH:mm:ss.SSSZ", doubles in Java Double.toString
// form (shortest digits via Ryu).  Same node model as the host serializer (host_serialize.cpp).
//
// Two passes, one lane per row: lengths (no stores) → exclusive scan on the stream → write at exact offsets, so the
// output is one contiguous blob copied to the host with a single D2H.  Bytes leave through the register-packed
// 16-B emitter (dxa_emit.h).  Every output table of a batch renders in the same launch pair (one segment each):
// one upload of the tables, one scan, one D2H of the lengths and one of the text per batch, not per output.
//
// The column tree is walked by a flat program the host derives from it (one FIELD op per node in preorder, a CLOSE
// op after each container's children, and for every FIELD the number of ops to jump when the field is omitted):
// no device recursion (call stacks live in scratch) and comma state is one bit per nesting level in a register.
// Strings are scanned 8 bytes at a time (SWAR test for bytes needing an escape).
#include "dxa_common.h"
#include "dxa_emit.h"
#include "dxa_ryu.h"

namespace {

enum Kind : int32_t {
  K_I64 = 0, K_F64 = 1, K_BOOL = 2, K_STR = 3, K_TS = 4, K_DATE = 5, K_CONST = 6, K_STRUCT = 7, K_MAP = 8,
  K_ARRAY = 9, K_RAW = 10, K_NULL = 11,
};

struct DevNode {
  int32_t kind, nchildren, child0, drop_nulls;
  int32_t name_off, name_len, const_off, const_len;   // into the text pool (names are pre-quoted JSON strings)
  const void* data;
  const uint8_t* valid;
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
};

// Several tables render in one launch pair: segment s owns rows [row[s], row[s+1]) of the output, render ops
// [pc[s], pc[s+1]) of the shared program and workgroups [block[s], block[s+1]) (a workgroup never straddles two
// segments, so the program a wave walks is uniform).  Row indices into a segment's columns are local to it.
constexpr int kMaxSeg = 16;

struct SerSegs {
  int32_t nseg;
  int32_t pad;
  int64_t row[kMaxSeg + 1];
  int32_t pc[kMaxSeg + 1];
  int32_t block[kMaxSeg + 1];
};

struct SerArgs {
  const DevNode* nodes;
  int32_t nnodes;
  const int32_t* prog;    // 4 ints per op: (code, node, depth, mode | skip << 8)
  int32_t nprog;
  const uint8_t* text;    // names and constants, each 8-B aligned and zero-padded (dxa/ops/serialize.py)
  int32_t text_words;
  int64_t* lens;          // length pass (line length incl. the newline)
  const int64_t* ends;    // write pass: inclusive scan of lens (line i starts at ends[i] - lens[i])
  uint8_t* out;
  SerSegs seg;
};

__constant__ uint64_t c_ryu_inv[2 * DXA_RYU_INV_TABLE_SIZE] = DXA_RYU_POW5_INV_SPLIT_INIT;
__constant__ uint64_t c_ryu_pos[2 * DXA_RYU_TABLE_SIZE] = DXA_RYU_POW5_SPLIT_INIT;

#define G1 __attribute__((address_space(1)))

// little-endian text constants for put_word
constexpr uint64_t kTrue = 0x65757274ull;          // "true"
constexpr uint64_t kFalse = 0x65736c6166ull;       // "false"
constexpr uint64_t kNull = 0x6c6c756eull;          // "null"
constexpr uint64_t kNaN = 0x224e614e22ull;         // "\"NaN\""
constexpr uint64_t kZeros = 0x3030303030303030ull; // "00000000"

__constant__ uint64_t c_pow10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                     100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                     1000000000000ull, 10000000000000ull, 100000000000000ull,
                                     1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                     1000000000000000000ull, 10000000000000000000ull};

// exactly nd (1..19) digits of x, zero-padded
template <bool W>
__device__ __forceinline__ void put_fixed64(dxa::Emitter<W>& e, uint64_t x, uint32_t nd) {
  if (nd > 16) {
    const uint64_t hi = x / 10000000000000000ull;
    e.put_fixed((uint32_t)hi, nd - 16);
    x -= hi * 10000000000000000ull;
    nd = 16;
  }
  if (nd > 8) {
    const uint64_t hi = x / 100000000ull;
    e.put_fixed((uint32_t)hi, nd - 8);
    e.put_fixed((uint32_t)(x - hi * 100000000ull), 8);
  } else {
    e.put_fixed((uint32_t)x, nd);
  }
}

template <bool W>
__device__ __forceinline__ void put_zeros(dxa::Emitter<W>& e, int k) {
  for (; k >= 8; k -= 8) e.put_word(kZeros, 8);
  if (k > 0) e.put_word(dxa::low_bytes(kZeros, (uint32_t)k), (uint32_t)k);
}

// x / 10^k for k in 1..17 and x < 10^17 without a 64-bit software division: double estimate, then exact correction
__device__ __forceinline__ uint64_t div_pow10(uint64_t x, int k) {
  const uint64_t p = c_pow10[k];
  uint64_t q = (uint64_t)((double)x / (double)p);
  while (q * p > x) --q;
  while ((q + 1) * p <= x) ++q;
  return q;
}

// Java Double.toString (the text of dxa::ryu::java_double) straight into the emitter: shortest digits from Ryu, then
// words of digits — no per-character buffer in scratch memory.
template <bool W>
__device__ __forceinline__ void put_java_double(dxa::Emitter<W>& e, double v) {
  if (v != v) { e.put_word(kNaN, 5); return; }                  // Spark's to_json quotes NaN / Infinity
  uint64_t bits;
  __builtin_memcpy(&bits, &v, 8);
  const bool neg = (bits >> 63) != 0;
  if ((bits & 0x7fffffffffffffffull) == 0x7ff0000000000000ull) {
    e.put('"');
    if (neg) e.put('-');
    e.put_word(0x7974696e69666e49ull, 8);                        // "Infinity"
    e.put('"');
    return;
  }
  if (neg) e.put('-');
  if ((bits & 0x7fffffffffffffffull) == 0) { e.put_word(0x302e30ull, 3); return; }   // "0.0"
  uint64_t d;
  int32_t ex;
  dxa::ryu::d2d(v, d, ex, c_ryu_inv, c_ryu_pos);
  const int len = (int)dxa::ryu::decimal_len(d);
  const int sci = ex + len - 1;
  if (sci >= -3 && sci < 7) {
    const int point = sci + 1;                                   // digits before the decimal point
    if (point <= 0) {
      e.put_word(0x2e30ull, 2);                                  // "0."
      put_zeros(e, -point);
      put_fixed64(e, d, (uint32_t)len);
    } else if (point >= len) {
      put_fixed64(e, d, (uint32_t)len);
      put_zeros(e, point - len);
      e.put_word(0x302eull, 2);                                  // ".0"
    } else {
      const uint64_t ip = div_pow10(d, len - point);
      put_fixed64(e, ip, (uint32_t)point);
      e.put('.');
      put_fixed64(e, d - ip * c_pow10[len - point], (uint32_t)(len - point));
    }
  } else {
    const uint64_t lead = len > 1 ? div_pow10(d, len - 1) : d;
    e.put((uint8_t)('0' + lead));
    e.put('.');
    if (len > 1) put_fixed64(e, d - lead * c_pow10[len - 1], (uint32_t)(len - 1));
    else e.put('0');
    e.put('E');
    int x = sci;
    if (x < 0) { e.put('-'); x = -x; }
    e.put_u32((uint32_t)x);
  }
}

__device__ __forceinline__ void dxa_civil(int64_t days, int64_t& y, unsigned& m, unsigned& d) {
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const unsigned doe = (unsigned)(days - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  y = (int64_t)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  if (m <= 2) ++y;
}

template <bool W>
__device__ __forceinline__ void put_date(dxa::Emitter<W>& e, int64_t days) {
  int64_t y; unsigned m, d;
  dxa_civil(days, y, m, d);
  if (y >= 0 && y < 10000) e.put_fixed((uint32_t)y, 4);
  else e.put_i64(y);
  e.put('-'); e.put2((int)m); e.put('-'); e.put2((int)d);
}

template <bool W>
__device__ __forceinline__ void put_ts(dxa::Emitter<W>& e, int64_t us) {
  const int64_t secs = us >= 0 ? us / 1000000 : -((-us + 999999) / 1000000);
  const int64_t frac = us - secs * 1000000;
  const int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  const int64_t sod = secs - days * 86400;
  e.put('"');
  put_date(e, days);
  e.put('T');
  e.put2((int)(sod / 3600)); e.put(':'); e.put2((int)(sod / 60 % 60)); e.put(':'); e.put2((int)(sod % 60));
  e.put('.');
  e.put_fixed((uint32_t)(frac / 1000), 3);
  e.put_word(0x225aull, 2);                                      // "Z\""
}

__device__ __forceinline__ uint64_t swar_has(uint64_t x, uint64_t pat) {
  const uint64_t v = x ^ pat;
  return (v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull;     // exact for the lowest flagged byte
}

// 8 bytes at s (aligned loads; an aligned word holding one byte of an allocation is inside it)
__device__ __forceinline__ uint64_t load8_any(const uint8_t* s) {
  const uint32_t o = (uint32_t)(reinterpret_cast<uintptr_t>(s) & 7);
  const G1 uint64_t* w = (const G1 uint64_t*)(s - o);
  const uint64_t lo = w[0];
  if (o == 0) return lo;
  return (lo >> (8 * o)) | (w[1] << (64 - 8 * o));
}

template <bool W>
__device__ __forceinline__ void put_escaped(dxa::Emitter<W>& e, uint32_t c) {
  uint64_t w;
  uint32_t n = 2;
  switch (c) {
    case '"': w = 0x225cull; break;
    case '\\': w = 0x5c5cull; break;
    case '\n': w = 0x6e5cull; break;
    case '\r': w = 0x725cull; break;
    case '\t': w = 0x745cull; break;
    case '\b': w = 0x625cull; break;
    case '\f': w = 0x665cull; break;
    default: {
      const uint32_t hi = c >> 4, lo = c & 15;
      w = 0x3030755cull | ((uint64_t)(hi < 10 ? '0' + hi : 'a' + hi - 10) << 32) |
          ((uint64_t)(lo < 10 ? '0' + lo : 'a' + lo - 10) << 40);            // \u00XY
      n = 6;
    }
  }
  e.put_word(w, n);
}

// JSON string: 8 bytes per step, SWAR test for bytes that need an escape; clean runs leave as whole words
template <bool W>
__device__ __forceinline__ void put_str(dxa::Emitter<W>& e, const uint8_t* s, int32_t n) {
  e.put('"');
  int32_t i = 0;
  while (i < n) {
    uint64_t x = load8_any(s + i);
    const int32_t avail = n - i < 8 ? n - i : 8;
    if (avail < 8) x = dxa::low_bytes(x, (uint32_t)avail) | (0x2020202020202020ull << (8 * avail));  // pad: clean
    const uint64_t m = ((x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull) |   // < 0x20
                       swar_has(x, 0x2222222222222222ull) | swar_has(x, 0x5C5C5C5C5C5C5C5Cull);
    int j = m ? (int)(__builtin_ctzll(m) >> 3) : 8;
    if (j > avail) j = avail;
    if (j) e.put_word(dxa::low_bytes(x, (uint32_t)j), (uint32_t)j);
    i += j;
    if (j < avail) {
      put_escaped(e, (uint32_t)((x >> (8 * j)) & 0xff));
      ++i;
    }
  }
  e.put('"');
}

// raw (already JSON) text from an arbitrary address
template <bool W>
__device__ __forceinline__ void put_raw(dxa::Emitter<W>& e, const uint8_t* s, int32_t n) {
  int32_t i = 0;
  for (; i + 8 <= n; i += 8) e.put_word(load8_any(s + i), 8);
  if (i < n) e.put_word(dxa::low_bytes(load8_any(s + i), (uint32_t)(n - i)), (uint32_t)(n - i));
}

enum : int32_t { P_FIELD = 0, P_CLOSE = 1 };
// FIELD modes: 0 struct member (omitted when null), 1 map member (null written), 2 array element (null written),
// 3 array element of a filterNull array (omitted when null)

// The render tables as the row loop reads them: staged in LDS per workgroup (uniform reads broadcast from LDS; from
// global memory the compiler must assume the output stores may alias them and re-issues every read as a vector load).
struct Tables {
  const int32_t* prog;
  const DevNode* nodes;
  const uint64_t* text64;
};

__device__ __forceinline__ Tables stage_tables(const SerArgs& a, uint64_t* smem) {
  const int node_words = a.nnodes * (int)(sizeof(DevNode) / 8);
  const int prog_words = (a.nprog * 4 + 1) / 2;
  const uint64_t* src_nodes = reinterpret_cast<const uint64_t*>(a.nodes);
  const uint64_t* src_prog = reinterpret_cast<const uint64_t*>(a.prog);
  const uint64_t* src_text = reinterpret_cast<const uint64_t*>(a.text);
  for (int q = threadIdx.x; q < node_words; q += blockDim.x) smem[q] = src_nodes[q];
  uint64_t* prog = smem + node_words;
  for (int q = threadIdx.x; q < prog_words; q += blockDim.x) prog[q] = src_prog[q];
  uint64_t* text = prog + prog_words;
  for (int q = threadIdx.x; q < a.text_words; q += blockDim.x) text[q] = src_text[q];
  __syncthreads();
  return Tables{reinterpret_cast<const int32_t*>(prog), reinterpret_cast<const DevNode*>(smem), text};
}

template <bool W>
__device__ __forceinline__ int64_t render_row(const Tables& t, int pc0, int pc1, int64_t row, uint8_t* dst) {
  dxa::Emitter<W> e(dst);
  e.put('{');
  uint32_t first = 1u;                                      // bit d: nothing written yet at nesting depth d
  for (int pc = pc0; pc < pc1; ++pc) {
    const int code = t.prog[4 * pc], nidx = t.prog[4 * pc + 1], depth = t.prog[4 * pc + 2], mw = t.prog[4 * pc + 3];
    const DevNode& nd = t.nodes[nidx];
    const int kind = nd.kind;
    if (code == P_CLOSE) {
      e.put(kind == K_ARRAY ? ']' : '}');
      continue;
    }
    const int mode = mw & 0xff;
    const int skip = mw >> 8;
    const bool null = kind == K_NULL || (nd.valid != nullptr && ((const G1 uint8_t*)nd.valid)[row] == 0);
    if (null && (mode == 0 || mode == 3)) { pc += skip; continue; }
    if (!((first >> depth) & 1u)) e.put(',');
    first &= ~(1u << depth);
    if (mode <= 1) e.put_text_words(t.text64 + (nd.name_off >> 3), nd.name_len);     // "name": (colon included)
    if (null) {
      e.put_word(kNull, 4);
      pc += skip;
      continue;
    }
    switch (kind) {
      case K_I64: e.put_i64(((const G1 int64_t*)nd.data)[row]); break;
      case K_F64: put_java_double(e, ((const G1 double*)nd.data)[row]); break;
      case K_BOOL:
        if (((const G1 uint8_t*)nd.data)[row]) e.put_word(kTrue, 4);
        else e.put_word(kFalse, 5);
        break;
      case K_STR: put_str(e, nd.arena + ((const G1 int64_t*)nd.starts)[row], ((const G1 int32_t*)nd.lens)[row]); break;
      case K_RAW: put_raw(e, nd.arena + ((const G1 int64_t*)nd.starts)[row], ((const G1 int32_t*)nd.lens)[row]); break;
      case K_TS: put_ts(e, ((const G1 int64_t*)nd.data)[row]); break;
      case K_DATE: e.put('"'); put_date(e, ((const G1 int64_t*)nd.data)[row]); e.put('"'); break;
      case K_CONST: e.put_text_words(t.text64 + (nd.const_off >> 3), nd.const_len); break;
      case K_STRUCT:
      case K_MAP:
      case K_ARRAY:
        e.put(kind == K_ARRAY ? '[' : '{');
        first |= 1u << (depth + 1);
        break;
      default: break;
    }
  }
  e.put_word(0x0a7dull, 2);                                 // "}\n"
  e.finish();
  return e.len;
}

// (segment, local row, global row) of this lane; false past the end of its segment
__device__ __forceinline__ bool seg_row(const SerSegs& g, int& s, int64_t& local, int64_t& row) {
  const int b = (int)blockIdx.x;
  s = 0;
  while (s + 1 < g.nseg && b >= g.block[s + 1]) ++s;      // uniform: at most kMaxSeg scalar compares
  local = (int64_t)(b - g.block[s]) * blockDim.x + threadIdx.x;
  row = g.row[s] + local;
  return row < g.row[s + 1];
}

__global__ __launch_bounds__(256) void ser_len_kernel(SerArgs a) {
  extern __shared__ uint64_t smem[];
  const Tables t = stage_tables(a, smem);
  int s;
  int64_t local, row;
  if (!seg_row(a.seg, s, local, row)) return;
  a.lens[row] = render_row<false>(t, a.seg.pc[s], a.seg.pc[s + 1], local, nullptr);
}

__global__ __launch_bounds__(256) void ser_write_kernel(SerArgs a) {
  extern __shared__ uint64_t smem[];
  const Tables t = stage_tables(a, smem);
  int s;
  int64_t local, row;
  if (!seg_row(a.seg, s, local, row)) return;
  render_row<true>(t, a.seg.pc[s], a.seg.pc[s + 1], local, a.out + (a.ends[row] - a.lens[row]));
}

size_t ser_lds_bytes(int32_t nnodes, int32_t nprog, int32_t text_words) {
  return (size_t)nnodes * sizeof(DevNode) + (size_t)((nprog * 4 + 1) / 2) * 8 + (size_t)text_words * 8;
}

constexpr size_t kMaxLds = 64 * 1024;

// Test entry: Java Double.toString of v[i] into a 32-byte slot — finite values through the serializer's word path
// (put_java_double), NaN / Infinity unquoted as the host formatter writes them.
__global__ __launch_bounds__(256) void java_double_kernel(const double* v, int64_t n, uint8_t* out, int32_t* lens) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = v[i];
  if (x != x || x - x != 0.0) {
    char buf[32];
    const int k = dxa::ryu::java_double(x, buf, c_ryu_inv, c_ryu_pos);
    for (int j = 0; j < k; ++j) out[32 * i + j] = (uint8_t)buf[j];
    lens[i] = k;
    return;
  }
  dxa::Emitter<true> e(out + 32 * i);
  put_java_double(e, x);
  e.finish();
  lens[i] = (int32_t)e.len;
}

const uint64_t h_ryu_inv[2 * DXA_RYU_INV_TABLE_SIZE] = DXA_RYU_POW5_INV_SPLIT_INIT;
const uint64_t h_ryu_pos[2 * DXA_RYU_TABLE_SIZE] = DXA_RYU_POW5_SPLIT_INIT;

}  // namespace

DXA_API int dxa_sernode_dev_size() { return (int)sizeof(DevNode); }

DXA_API int dxa_sersegs_size() { return (int)sizeof(SerSegs); }
DXA_API int dxa_sersegs_max() { return kMaxSeg; }

// One pass of the serializer over every segment.  `tables` holds the node array (nnodes DevNode), then the flat
// render program (nprog ops of 4 ints, padded to 8 B), then the text pool (text_words 8-B words; names / constants
// 8-B aligned and zero-padded) — one upload per batch, built by dxa/ops/serialize.py.  `segs` is a host SerSegs with
// nseg, row[0..nseg] and pc[0..nseg] filled; the workgroup ranges are derived here.  The tables are staged in LDS,
// so they must fit in 64 KiB together.  write == 0: line lengths into `lens`; write == 1: lines into `out` at
// ends[i] - lens[i].
DXA_API int dxa_serialize_rows(int32_t write, const void* tables, int32_t nnodes, int32_t nprog, int32_t text_words,
                               const void* segs, int64_t* lens, const int64_t* ends, uint8_t* out, void* st) {
  SerSegs g = *(const SerSegs*)segs;
  if (g.nseg <= 0 || g.nseg > kMaxSeg) return (int)hipErrorInvalidValue;
  int64_t blocks = 0;
  for (int s = 0; s < g.nseg; ++s) {
    if (g.row[s + 1] < g.row[s] || g.pc[s + 1] < g.pc[s] || g.pc[s + 1] > nprog) return (int)hipErrorInvalidValue;
    g.block[s] = (int32_t)blocks;
    blocks += (g.row[s + 1] - g.row[s] + 255) / 256;
  }
  g.block[g.nseg] = (int32_t)blocks;
  if (blocks == 0) return 0;
  if (blocks > 0x7fffffff) return (int)hipErrorInvalidValue;
  const size_t lds = ser_lds_bytes(nnodes, nprog, text_words);
  if (lds > kMaxLds) return (int)hipErrorInvalidValue;
  const uint8_t* base = (const uint8_t*)tables;
  const size_t prog_off = (size_t)nnodes * sizeof(DevNode);
  const size_t text_off = prog_off + (size_t)((nprog * 4 + 1) / 2) * 8;
  SerArgs a{(const DevNode*)base, nnodes, (const int32_t*)(base + prog_off), nprog, base + text_off, text_words,
            lens, ends, out, g};
  if (write)
    hipLaunchKernelGGL(ser_write_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)st, a);
  else hipLaunchKernelGGL(ser_len_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

// Device Java-double formatting into 32-byte slots (tests compare it with the host formatter).
DXA_API int dxa_java_double_dev(const double* v, int64_t n, uint8_t* out, int32_t* lens, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(java_double_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st, v, n,
                     out, lens);
  return (int)hipGetLastError();
}

// The same __host__ __device__ formatter run on the CPU (no GPU needed) — lets CPU tests pin the device algorithm.
DXA_API int dxa_java_double_hostcheck(const double* v, int64_t n, uint8_t* out, int32_t* lens) {
  for (int64_t i = 0; i < n; ++i) {
    char buf[32];
    const int k = dxa::ryu::java_double(v[i], buf, h_ryu_inv, h_ryu_pos);
    for (int j = 0; j < k; ++j) out[32 * i + j] = (uint8_t)buf[j];
    lens[i] = k;
  }
  return 0;
}

// CAST(double AS STRING): Java Double.toString text (Spark's cast), two passes — lengths, then bytes at the
// host-scanned offsets.  Invalid rows get length 0.
namespace {
__global__ void f64_str_len_kernel(const double* __restrict__ v, const uint8_t* __restrict__ valid, int64_t n,
                                   int64_t* __restrict__ out_len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out_len[i] = (valid && !valid[i]) ? 0 : dxa::ryu::java_double(v[i], nullptr, c_ryu_inv, c_ryu_pos);
}

__global__ void f64_str_write_kernel(const double* __restrict__ v, const uint8_t* __restrict__ valid, int64_t n,
                                     const int64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) continue;
    char buf[32];
    const int l = dxa::ryu::java_double(v[i], buf, c_ryu_inv, c_ryu_pos);
    for (int k = 0; k < l; ++k) dst[off[i] + k] = (uint8_t)buf[k];
  }
}
}  // namespace

DXA_API int dxa_f64_str_len(const double* v, const uint8_t* valid, int64_t n, int64_t* out_len, void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(f64_str_len_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, valid, n,
                     out_len);
  return (int)hipGetLastError();
}

DXA_API int dxa_f64_str_write(const double* v, const uint8_t* valid, int64_t n, const int64_t* off, uint8_t* dst,
                              void* st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(f64_str_write_kernel, dim3(dxa_blocks(n, 256)), dim3(256), 0, (hipStream_t)st, v, valid, n,
                     off, dst);
  return (int)hipGetLastError();
}
