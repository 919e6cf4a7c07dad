// Device JSON-lines serializer (kernel K20): rows of a columnar table → newline-terminated JSON with
// Spark ``to_json(struct(*))`` semantics — field order = column order, null fields omitted, MAP nulls written as
// null, filterNull arrays skip nulls, timestamps as "yyyy-MM-dd'T'HH:mm:ss.SSSZ", doubles in Java Double.toString
// form (shortest digits via Ryu).  Same node model as the host serializer (host_serialize.cpp).
//
// Two passes, one lane per row: lengths (no stores) → exclusive scan on the stream → write at exact offsets, so the
// output is one contiguous blob copied to the host with a single D2H.  Bytes leave through the register-packed
// 16-B emitter (dxa_emit.h).
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
  const int32_t* top;
  int32_t ntop;
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
__device__ __forceinline__ void put_text(dxa::Emitter<W>& e, const uint8_t* s, int n) {
  for (int i = 0; i < n; ++i) e.put(s[i]);
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

template <bool W>
__device__ void put_str(dxa::Emitter<W>& e, const uint8_t* s, int32_t n) {
  e.put('"');
  for (int32_t i = 0; i < n; ++i) {
    const uint8_t c = s[i];
    if (c >= 0x20 && c != '"' && c != '\\') { e.put(c); continue; }
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
        const char* hex = "0123456789abcdef";
        e.put('u'); e.put('0'); e.put('0'); e.put((uint8_t)hex[c >> 4]); e.put((uint8_t)hex[c & 15]);
      }
    }
  }
  e.put('"');
}

template <bool W>
__device__ void put_double(dxa::Emitter<W>& e, double v) {
  // NaN / Infinity are JSON strings in Spark's to_json
  if (v != v) { put_text(e, (const uint8_t*)"\"NaN\"", 5); return; }
  char buf[32];
  const int n = dxa::ryu::java_double(v, buf, c_ryu_inv, c_ryu_pos);
  const bool inf = buf[n - 1] == 'y';
  if (inf) e.put('"');
  for (int i = 0; i < n; ++i) e.put((uint8_t)buf[i]);
  if (inf) e.put('"');
}

template <bool W>
__device__ void put_value(dxa::Emitter<W>& e, const SerArgs& a, const DevNode& nd, int64_t row, int depth);

template <bool W>
__device__ void put_children(dxa::Emitter<W>& e, const SerArgs& a, const DevNode& nd, int64_t row, int depth) {
  const bool is_array = nd.kind == K_ARRAY;
  e.put(is_array ? '[' : '{');
  bool first = true;
  for (int c = 0; c < nd.nchildren; ++c) {
    const DevNode& ch = a.nodes[nd.child0 + c];
    const bool null = is_null(ch, row);
    if (null && (nd.kind == K_STRUCT || (is_array && nd.drop_nulls))) continue;
    if (!first) e.put(',');
    first = false;
    if (!is_array) {
      put_text(e, a.text + ch.name_off, ch.name_len);
      e.put(':');
    }
    if (null) put_text(e, (const uint8_t*)"null", 4);
    else put_value(e, a, ch, row, depth + 1);
  }
  e.put(is_array ? ']' : '}');
}

template <bool W>
__device__ void put_value(dxa::Emitter<W>& e, const SerArgs& a, const DevNode& nd, int64_t row, int depth) {
  switch (nd.kind) {
    case K_I64: put_i64(e, ((const int64_t*)nd.data)[row]); break;
    case K_F64: put_double(e, ((const double*)nd.data)[row]); break;
    case K_BOOL:
      if (((const uint8_t*)nd.data)[row]) put_text(e, (const uint8_t*)"true", 4);
      else put_text(e, (const uint8_t*)"false", 5);
      break;
    case K_STR: put_str(e, nd.arena + nd.starts[row], nd.lens[row]); break;
    case K_RAW: put_text(e, nd.arena + nd.starts[row], nd.lens[row]); break;
    case K_TS: put_ts(e, ((const int64_t*)nd.data)[row]); break;
    case K_DATE: e.put('"'); put_date(e, ((const int64_t*)nd.data)[row]); e.put('"'); break;
    case K_CONST: put_text(e, a.text + nd.const_off, nd.const_len); break;
    case K_STRUCT:
    case K_MAP:
    case K_ARRAY:
      if (depth < 16) put_children(e, a, nd, row, depth);
      break;
    default: break;
  }
}

template <bool W>
__device__ int64_t render_row(const SerArgs& a, int64_t row, uint8_t* dst) {
  dxa::Emitter<W> e(dst);
  e.put('{');
  bool first = true;
  for (int t = 0; t < a.ntop; ++t) {
    const DevNode& nd = a.nodes[a.top[t]];
    if (is_null(nd, row)) continue;
    if (!first) e.put(',');
    first = false;
    put_text(e, a.text + nd.name_off, nd.name_len);
    e.put(':');
    put_value(e, a, nd, row, 0);
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

__global__ __launch_bounds__(256) void ser_write_kernel(SerArgs a) {
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

DXA_API int dxa_serialize_lengths(const void* nodes, const int32_t* top, int32_t ntop, const uint8_t* text, int64_t n,
                                  int64_t* lens, void* st) {
  if (n <= 0) return 0;
  SerArgs a{(const DevNode*)nodes, top, ntop, text, n, lens, nullptr, nullptr};
  hipLaunchKernelGGL(ser_len_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)st, a);
  return (int)hipGetLastError();
}

DXA_API int dxa_serialize_write(const void* nodes, const int32_t* top, int32_t ntop, const uint8_t* text, int64_t n,
                                const int64_t* offs, uint8_t* out, void* st) {
  if (n <= 0) return 0;
  SerArgs a{(const DevNode*)nodes, top, ntop, text, n, nullptr, offs, out};
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
