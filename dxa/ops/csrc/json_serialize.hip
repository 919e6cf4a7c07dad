// Device JSON-lines serializer (kernel K20): rows of a columnar table → newline-terminated JSON with
// Spark ``to_json(struct(*))`` semantics — field order = column order, null fields omitted, MAP nulls written as
// null, filterNull arrays skip nulls, timestamps as "yyyy-MM-dd'T'HH:mm:ss.SSSZ", doubles in Java Double.toString
// form (shortest digits via Ryu).  Same node model as the host serializer (host_serialize.cpp).
//
// Two passes, one lane per row: lengths (no stores) → exclusive scan on the stream → write at exact offsets, so the
// output is one contiguous blob copied to the host with a single D2H.  Bytes leave through the register-packed
// 16-B emitter (dxa_emit.h).
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

struct SerArgs {
  const DevNode* nodes;
  const int32_t* prog;    // 4 ints per op: (code, node, depth, mode | skip << 8)
  int32_t nprog;
  const uint8_t* text;
  int64_t n;
  int64_t* lens;          // length pass (line length incl. the newline)
  const int64_t* offs;    // write pass
  uint8_t* out;
};

__constant__ uint64_t c_ryu_inv[2 * DXA_RYU_INV_TABLE_SIZE] = DXA_RYU_POW5_INV_SPLIT_INIT;
__constant__ uint64_t c_ryu_pos[2 * DXA_RYU_TABLE_SIZE] = DXA_RYU_POW5_SPLIT_INIT;

__device__ __forceinline__ bool is_null(const DevNode& nd, int64_t row) {
  if (nd.kind == K_NULL) return true;
  return nd.valid != nullptr && nd.valid[row] == 0;
}


template <bool W>
__device__ void put_u64(dxa::Emitter<W>& e, uint64_t v) {
  uint64_t p = 1;
  while (v / p >= 10) p *= 10;
  for (; p; p /= 10) e.put((uint8_t)('0' + (v / p) % 10));
}

template <bool W>
__device__ void put_i64(dxa::Emitter<W>& e, int64_t v) {
  if (v < 0) { e.put('-'); put_u64(e, 0ull - (uint64_t)v); } else put_u64(e, (uint64_t)v);
}

template <bool W>
__device__ __forceinline__ void put2(dxa::Emitter<W>& e, unsigned v) {
  e.put((uint8_t)('0' + v / 10));
  e.put((uint8_t)('0' + v % 10));
}

__device__ void civil(int64_t days, int64_t& y, unsigned& m, unsigned& d) {
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
__device__ void put_date(dxa::Emitter<W>& e, int64_t days) {
  int64_t y; unsigned m, d;
  civil(days, y, m, d);
  if (y >= 0 && y < 10000) {
    e.put((uint8_t)('0' + y / 1000)); e.put((uint8_t)('0' + y / 100 % 10));
    e.put((uint8_t)('0' + y / 10 % 10)); e.put((uint8_t)('0' + y % 10));
  } else {
    put_i64(e, y);
  }
  e.put('-'); put2(e, m); e.put('-'); put2(e, d);
}

template <bool W>
__device__ void put_ts(dxa::Emitter<W>& e, int64_t us) {
  const int64_t secs = us >= 0 ? us / 1000000 : -((-us + 999999) / 1000000);
  const int64_t frac = us - secs * 1000000;
  const int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  const int64_t sod = secs - days * 86400;
  e.put('"');
  put_date(e, days);
  e.put('T');
  put2(e, (unsigned)(sod / 3600)); e.put(':'); put2(e, (unsigned)(sod / 60 % 60)); e.put(':');
  put2(e, (unsigned)(sod % 60));
  e.put('.');
  const unsigned ms = (unsigned)(frac / 1000);
  e.put((uint8_t)('0' + ms / 100)); e.put((uint8_t)('0' + ms / 10 % 10)); e.put((uint8_t)('0' + ms % 10));
  e.put('Z'); e.put('"');
}

#define G1 __attribute__((address_space(1)))

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
  e.put('\\');
  switch (c) {
    case '"': e.put('"'); break;
    case '\\': e.put('\\'); break;
    case '\n': e.put('n'); break;
    case '\r': e.put('r'); break;
    case '\t': e.put('t'); break;
    case '\b': e.put('b'); break;
    case '\f': e.put('f'); break;
    default: {
      const uint32_t hi = c >> 4, lo = c & 15;
      e.put('u'); e.put('0'); e.put('0');
      e.put((uint8_t)(hi < 10 ? '0' + hi : 'a' + hi - 10));
      e.put((uint8_t)(lo < 10 ? '0' + lo : 'a' + lo - 10));
    }
  }
}

template <bool W>
__device__ void put_str(dxa::Emitter<W>& e, const uint8_t* s, int32_t n) {
  e.put('"');
  int32_t i = 0;
  while (i + 8 <= n) {                                       // 8 bytes per step: escape test by SWAR
    const uint64_t x = load8_any(s + i);
    const uint64_t m = ((x - 0x2020202020202020ull) & ~x & 0x8080808080808080ull) |   // < 0x20
                       swar_has(x, 0x2222222222222222ull) | swar_has(x, 0x5C5C5C5C5C5C5C5Cull);
    const int j = m ? (int)(__builtin_ctzll(m) >> 3) : 8;
    for (int t = 0; t < j; ++t) e.put((uint8_t)(x >> (8 * t)));
    i += j;
    if (j < 8) {
      put_escaped(e, (uint32_t)((x >> (8 * j)) & 0xff));
      ++i;
    }
  }
  for (; i < n; ++i) {
    const uint32_t c = ((const G1 uint8_t*)s)[i];
    if (c >= 0x20 && c != '"' && c != '\\') e.put((uint8_t)c);
    else put_escaped(e, c);
  }
  e.put('"');
}

template <bool W>
__device__ void put_double(dxa::Emitter<W>& e, double v) {
  // NaN / Infinity are JSON strings in Spark's to_json
  if (v != v) { e.put('"'); e.put('N'); e.put('a'); e.put('N'); e.put('"'); return; }
  char buf[32];
  const int n = dxa::ryu::java_double(v, buf, c_ryu_inv, c_ryu_pos);
  const bool inf = buf[n - 1] == 'y';
  if (inf) e.put('"');
  for (int i = 0; i < n; ++i) e.put((uint8_t)buf[i]);
  if (inf) e.put('"');
}

enum : int32_t { P_FIELD = 0, P_CLOSE = 1 };
// FIELD modes: 0 struct member (omitted when null), 1 map member (null written), 2 array element (null written),
// 3 array element of a filterNull array (omitted when null)

template <bool W>
__device__ __forceinline__ void put_text(dxa::Emitter<W>& e, const G1 uint8_t* s, int n) {
  for (int i = 0; i < n; ++i) e.put(s[i]);
}

template <bool W>
__device__ int64_t render_row(const SerArgs& a, int64_t row, uint8_t* dst) {
  dxa::Emitter<W> e(dst);
  const G1 int32_t* prog = (const G1 int32_t*)a.prog;
  const G1 DevNode* nodes = (const G1 DevNode*)a.nodes;
  const G1 uint8_t* text = (const G1 uint8_t*)a.text;
  e.put('{');
  uint32_t first = 1u;                                      // bit d: nothing written yet at nesting depth d
  for (int pc = 0; pc < a.nprog; ++pc) {
    // four separate loads: copying an int4 (HIP vector class) out of an address-space-1 pointer drops lanes
    const int code = prog[4 * pc], nidx = prog[4 * pc + 1], depth = prog[4 * pc + 2], mw = prog[4 * pc + 3];
    if (code == P_CLOSE) {
      e.put(nodes[nidx].kind == K_ARRAY ? ']' : '}');
      continue;
    }
    const int mode = mw & 0xff;
    const int skip = mw >> 8;
    const G1 DevNode& nd = nodes[nidx];
    const int kind = nd.kind;
    const bool null = kind == K_NULL || (nd.valid != nullptr && ((const G1 uint8_t*)nd.valid)[row] == 0);
    if (null && (mode == 0 || mode == 3)) { pc += skip; continue; }
    if (!((first >> depth) & 1u)) e.put(',');
    first &= ~(1u << depth);
    if (mode <= 1) {
      put_text(e, text + nd.name_off, nd.name_len);
      e.put(':');
    }
    if (null) {
      e.put('n'); e.put('u'); e.put('l'); e.put('l');
      pc += skip;
      continue;
    }
    switch (kind) {
      case K_I64: put_i64(e, ((const G1 int64_t*)nd.data)[row]); break;
      case K_F64: put_double(e, ((const G1 double*)nd.data)[row]); break;
      case K_BOOL:
        if (((const G1 uint8_t*)nd.data)[row]) { e.put('t'); e.put('r'); e.put('u'); e.put('e'); }
        else { e.put('f'); e.put('a'); e.put('l'); e.put('s'); e.put('e'); }
        break;
      case K_STR: put_str(e, nd.arena + ((const G1 int64_t*)nd.starts)[row], ((const G1 int32_t*)nd.lens)[row]); break;
      case K_RAW:
        put_text(e, (const G1 uint8_t*)nd.arena + ((const G1 int64_t*)nd.starts)[row],
                 ((const G1 int32_t*)nd.lens)[row]);
        break;
      case K_TS: put_ts(e, ((const G1 int64_t*)nd.data)[row]); break;
      case K_DATE: e.put('"'); put_date(e, ((const G1 int64_t*)nd.data)[row]); e.put('"'); break;
      case K_CONST: put_text(e, text + nd.const_off, nd.const_len); break;
      case K_STRUCT:
      case K_MAP:
      case K_ARRAY:
        e.put(kind == K_ARRAY ? '[' : '{');
        first |= 1u << (depth + 1);
        break;
      default: break;
    }
  }
  e.put('}');
  e.put('\n');
  e.finish();
  return e.len;
}

__global__ __launch_bounds__(256) void ser_len_kernel(SerArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  a.lens[i] = render_row<false>(a, i, nullptr);
}

// amdgpu_waves_per_eu(4): 127 VGPRs instead of 151 (4 waves per SIMD instead of 3), no extra scratch.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void ser_write_kernel(SerArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  render_row<true>(a, i, a.out + a.offs[i]);
}

__global__ __launch_bounds__(256) void java_double_kernel(const double* v, int64_t n, uint8_t* out, int32_t* lens) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  char buf[32];
  const int k = dxa::ryu::java_double(v[i], buf, c_ryu_inv, c_ryu_pos);
  for (int j = 0; j < k; ++j) out[32 * i + j] = (uint8_t)buf[j];
  lens[i] = k;
}

const uint64_t h_ryu_inv[2 * DXA_RYU_INV_TABLE_SIZE] = DXA_RYU_POW5_INV_SPLIT_INIT;
const uint64_t h_ryu_pos[2 * DXA_RYU_TABLE_SIZE] = DXA_RYU_POW5_SPLIT_INIT;

}  // namespace

DXA_API int dxa_sernode_dev_size() { return (int)sizeof(DevNode); }

// `prog` / `nprog`: the flat render program (4 ints per op) built by dxa/ops/serialize.py from the node tree.
DXA_API int dxa_serialize_lengths(const void* nodes, const int32_t* prog, int32_t nprog, const uint8_t* text, int64_t n,
                                  int64_t* lens, void* st) {
  if (n <= 0) return 0;
  SerArgs a{(const DevNode*)nodes, prog, nprog, text, n, lens, nullptr, nullptr};
  hipLaunchKernelGGL(ser_len_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

DXA_API int dxa_serialize_write(const void* nodes, const int32_t* prog, int32_t nprog, const uint8_t* text, int64_t n,
                                const int64_t* offs, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  SerArgs a{(const DevNode*)nodes, prog, nprog, text, n, nullptr, offs, out};
  hipLaunchKernelGGL(ser_write_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st, a);
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
