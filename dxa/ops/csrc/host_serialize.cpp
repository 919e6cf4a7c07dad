// Native host-side JSON row serialiser (Spark `to_json(struct(*))` semantics) for sink egress.
//
// Reference behaviour: DataProcessing/datax-host/src/main/scala/datax/sink/OutputManager.scala:116-118 — field order
// = column order, null struct fields omitted (map values keep `null`), doubles rendered like Java
// Double.toString (shortest round-trip digits; plain notation for 1e-3 <= |x| < 1e7, else d.dddE±n), timestamps
// `yyyy-MM-dd'T'HH:mm:ss.SSS'Z'` (UTC), `filterNull` arrays skip null elements, raw JSON values verbatim.
//
// Rows are split across worker threads; each renders into a private buffer, then buffers are stitched into one
// newline-separated blob the sinks write as-is.
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {

struct SerNode {
  int32_t kind;        // see Kind
  int32_t nchildren;   // struct/map/array
  int32_t child0;      // index of first child in the node array (children are contiguous)
  int32_t drop_nulls;  // array: skip null elements
  const char* name;    // pre-escaped, quoted field name (children of struct/map, and top-level columns)
  int32_t name_len;
  int32_t pad;
  const void* data;    // i64 / f64 / u8 values
  const uint8_t* valid;
  const uint8_t* arena;
  const int64_t* starts;
  const int32_t* lens;
  const char* const_text;  // constant pre-rendered JSON value
  int32_t const_len;
  int32_t pad2;
};
}

namespace {

enum Kind : int32_t {
  K_I64 = 0, K_F64 = 1, K_BOOL = 2, K_STR = 3, K_TS = 4, K_DATE = 5, K_CONST = 6, K_STRUCT = 7, K_MAP = 8,
  K_ARRAY = 9, K_RAW = 10, K_NULL = 11,
};

void put_i64(std::string& o, int64_t v) {
  char b[24];
  auto r = std::to_chars(b, b + 24, v);
  o.append(b, r.ptr);
}

void put_java_double(std::string& o, double d) {
  if (d != d) { o += "\"NaN\""; return; }
  if (d == __builtin_inf()) { o += "\"Infinity\""; return; }
  if (d == -__builtin_inf()) { o += "\"-Infinity\""; return; }
  if (d == 0.0) { o += std::signbit(d) ? "-0.0" : "0.0"; return; }
  char b[64];
  auto r = std::to_chars(b, b + 64, d, std::chars_format::scientific);
  // b = [-]D[.DDDD]e±XX
  const char* p = b;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[32];
  int nd = 0;
  const char* e = p;
  while (e < r.ptr && *e != 'e') {
    if (*e != '.') digits[nd++] = *e;
    ++e;
  }
  int exp10 = 0;
  std::from_chars(e + 1 + (e[1] == '+'), r.ptr, exp10);
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  if (neg) o += '-';
  const double a = neg ? -d : d;
  if (a >= 1e-3 && a < 1e7) {
    const int point = exp10 + 1;  // digits before the decimal point
    if (point <= 0) {
      o += "0.";
      for (int i = 0; i < -point; ++i) o += '0';
      o.append(digits, nd);
    } else if (point >= nd) {
      o.append(digits, nd);
      for (int i = nd; i < point; ++i) o += '0';
      o += ".0";
    } else {
      o.append(digits, point);
      o += '.';
      o.append(digits + point, nd - point);
    }
  } else {
    o += digits[0];
    o += '.';
    if (nd > 1) o.append(digits + 1, nd - 1); else o += '0';
    o += 'E';
    put_i64(o, exp10);
  }
}

void civil(int64_t days, int64_t& y, unsigned& m, unsigned& d) {
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

void put2(std::string& o, unsigned v) { o += (char)('0' + v / 10); o += (char)('0' + v % 10); }

void put_date(std::string& o, int64_t days) {
  int64_t y; unsigned m, d;
  civil(days, y, m, d);
  char b[8];
  std::snprintf(b, sizeof b, "%04lld", (long long)y);
  o += b; o += '-'; put2(o, m); o += '-'; put2(o, d);
}

void put_ts(std::string& o, int64_t us) {
  int64_t secs = us >= 0 ? us / 1000000 : -((-us + 999999) / 1000000);
  int64_t frac = us - secs * 1000000;
  int64_t days = secs >= 0 ? secs / 86400 : -((-secs + 86399) / 86400);
  int64_t sod = secs - days * 86400;
  o += '"';
  put_date(o, days);
  o += 'T';
  put2(o, (unsigned)(sod / 3600)); o += ':'; put2(o, (unsigned)(sod / 60 % 60)); o += ':'; put2(o, (unsigned)(sod % 60));
  o += '.';
  const unsigned ms = (unsigned)(frac / 1000);
  o += (char)('0' + ms / 100); o += (char)('0' + ms / 10 % 10); o += (char)('0' + ms % 10);
  o += "Z\"";
}

void put_str(std::string& o, const uint8_t* s, int32_t n) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  for (int32_t i = 0; i < n; ++i) {
    const uint8_t c = s[i];
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c < 0x20) { o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15]; }
        else o += (char)c;
    }
  }
  o += '"';
}

// returns false when the value is null (nothing appended)
bool put_value(std::string& o, const SerNode* nodes, const SerNode& n, int64_t row) {
  if (n.valid && !n.valid[row]) return false;
  switch (n.kind) {
    case K_I64: put_i64(o, ((const int64_t*)n.data)[row]); return true;
    case K_F64: put_java_double(o, ((const double*)n.data)[row]); return true;
    case K_BOOL: o += ((const uint8_t*)n.data)[row] ? "true" : "false"; return true;
    case K_STR: put_str(o, n.arena + n.starts[row], n.lens[row]); return true;
    case K_RAW: o.append((const char*)n.arena + n.starts[row], n.lens[row]); return true;
    case K_TS: put_ts(o, ((const int64_t*)n.data)[row]); return true;
    case K_DATE: o += '"'; put_date(o, ((const int64_t*)n.data)[row]); o += '"'; return true;
    case K_CONST: o.append(n.const_text, n.const_len); return true;
    case K_NULL: return false;
    case K_STRUCT:
    case K_MAP: {
      o += '{';
      bool first = true;
      for (int c = 0; c < n.nchildren; ++c) {
        const SerNode& ch = nodes[n.child0 + c];
        const size_t mark = o.size();
        if (!first) o += ',';
        o.append(ch.name, ch.name_len);
        o += ':';
        if (put_value(o, nodes, ch, row)) { first = false; continue; }
        if (n.kind == K_MAP) { o += "null"; first = false; continue; }
        o.resize(mark);
      }
      o += '}';
      return true;
    }
    case K_ARRAY: {
      o += '[';
      bool first = true;
      for (int c = 0; c < n.nchildren; ++c) {
        const SerNode& ch = nodes[n.child0 + c];
        const size_t mark = o.size();
        if (!first) o += ',';
        if (put_value(o, nodes, ch, row)) { first = false; continue; }
        if (n.drop_nulls) { o.resize(mark); continue; }
        o += "null";
        first = false;
      }
      o += ']';
      return true;
    }
  }
  return false;
}

void render_rows(const SerNode* nodes, const int32_t* top, int32_t ntop, int64_t r0, int64_t r1, std::string& o,
                 int64_t* line_len) {
  for (int64_t r = r0; r < r1; ++r) {
    const size_t start = o.size();
    o += '{';
    bool first = true;
    for (int t = 0; t < ntop; ++t) {
      const SerNode& n = nodes[top[t]];
      const size_t mark = o.size();
      if (!first) o += ',';
      o.append(n.name, n.name_len);
      o += ':';
      if (put_value(o, nodes, n, r)) first = false; else o.resize(mark);
    }
    o += '}';
    line_len[r] = (int64_t)(o.size() - start);
    o += '\n';
  }
}

}  // namespace

extern "C" {

// Serialise nrows rows. Returns a malloc'd blob (caller frees with dxa_host_free) of newline-terminated JSON lines;
// *out_len receives its size; line_len[r] receives each line's length (without the newline).
__attribute__((visibility("default"))) char* dxa_serialize_rows(const SerNode* nodes, int32_t nnodes,
                                                                const int32_t* top, int32_t ntop, int64_t nrows,
                                                                int32_t nthreads, int64_t* line_len,
                                                                int64_t* out_len) {
  (void)nnodes;
  if (nthreads < 1) nthreads = 1;
  if (nrows < 4096) nthreads = 1;
  std::vector<std::string> parts((size_t)nthreads);
  std::vector<std::thread> ths;
  const int64_t chunk = (nrows + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t r0 = t * chunk, r1 = std::min<int64_t>(nrows, r0 + chunk);
    if (r0 >= r1) break;
    auto fn = [&, t, r0, r1] {
      parts[t].reserve((size_t)(r1 - r0) * 128);
      render_rows(nodes, top, ntop, r0, r1, parts[t], line_len);
    };
    if (t == nthreads - 1 || nthreads == 1) fn(); else ths.emplace_back(fn);
  }
  for (auto& th : ths) th.join();
  size_t total = 0;
  for (auto& p : parts) total += p.size();
  char* out = (char*)std::malloc(total ? total : 1);
  size_t off = 0;
  for (auto& p : parts) { std::memcpy(out + off, p.data(), p.size()); off += p.size(); }
  *out_len = (int64_t)total;
  return out;
}

__attribute__((visibility("default"))) void dxa_host_free(void* p) { std::free(p); }

__attribute__((visibility("default"))) int dxa_sernode_size() { return (int)sizeof(SerNode); }

__attribute__((visibility("default"))) int dxa_java_double(double d, char* out, int cap) {
  std::string s;
  put_java_double(s, d);
  const int n = (int)std::min<size_t>(s.size(), (size_t)cap);
  std::memcpy(out, s.data(), n);
  return n;
}
}
