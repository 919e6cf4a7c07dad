// CSV / TSV reference data → device string columns (the reference loads reference data with Spark's CSV reader,
// datax-utility/.../CSVUtil.scala:15-41: delimiter option, header option, every column a string).
//
// The file's bytes are framed into lines on the device first (newline-framing kernels in strings.hip; Spark's
// default multiLine=false, so a newline always ends a record).  This kernel then tokenizes one line per lane:
// fields are [start, len) views into the same byte arena, so a 100 M-row table costs one pass over its bytes plus
// 13 B of field descriptors per cell, and no host round trip.  Semantics (Spark 2.4 CSV, PERMISSIVE):
//   * a trailing '\r' is dropped (CRLF files);
//   * a field starting with the quote char is quoted: it ends at the next unescaped quote; inside it the escape char
//     (default '\\') or a doubled quote yields one literal quote (the bytes are rewritten in place, left-compacted,
//     so the field stays one contiguous view); characters between the closing quote and the delimiter are dropped;
//   * an empty unquoted field is null (nullValue ""), an empty quoted field ("") is the empty string;
//   * missing trailing fields are null, extra fields are dropped.
// Lines are read through a 32-byte register window (two aligned 16-B loads), so most lines cost one or two loads.
#include "dxa_common.h"

namespace {

struct LineWin {
  const uint8_t* base;
  int64_t wb;
  uint4 a, b;
  __device__ __forceinline__ uint32_t at(int64_t q) {
    if (q - wb >= 32 || q < wb) {
      const uintptr_t addr = reinterpret_cast<uintptr_t>(base + q);
      wb = q - (int64_t)(addr & 15);
      const uint4* w = reinterpret_cast<const uint4*>(base + wb);
      a = w[0];
      b = w[1];
    }
    const uint32_t o = (uint32_t)(q - wb);
    return o < 16 ? dxa::window_byte(a, o) : dxa::window_byte(b, o - 16);
  }
};

__global__ __launch_bounds__(256) void csv_tokenize_kernel(uint8_t* __restrict__ buf, const int64_t* __restrict__ offs,
                                                           int64_t nlines, int32_t ncols, uint32_t delim,
                                                           uint32_t quote, uint32_t escape,
                                                           int64_t* __restrict__ starts, int32_t* __restrict__ lens,
                                                           uint8_t* __restrict__ valid, uint8_t* __restrict__ row_ok) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nlines) return;
  int64_t p = offs[i];
  int64_t end = offs[i + 1];
  LineWin w{buf, -64, make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  // a framed record may carry the newlines of empty lines dropped after it, and CRLF ends
  while (end > p && (w.at(end - 1) == '\n' || w.at(end - 1) == '\r')) --end;
  row_ok[i] = end > p ? 1 : 0;                       // whitespace-only lines are skipped, as Spark does
  bool more = true;                      // a field starts at p (a line always has at least one)
  for (int32_t j = 0; j < ncols; ++j) {
    const int64_t o = (int64_t)j * nlines + i;
    if (!more) {                          // missing trailing field
      starts[o] = 0;
      lens[o] = 0;
      valid[o] = 0;
      continue;
    }
    if (p < end && w.at(p) == quote) {
      const int64_t f = p + 1;
      int64_t q = f, out = f;
      bool rewrite = false;
      while (q < end) {
        const uint32_t c = w.at(q);
        if (c == escape && escape != quote && q + 1 < end) {
          const uint32_t nx = w.at(q + 1);
          if (nx == quote || nx == escape) {
            buf[out] = (uint8_t)nx;
            rewrite = true;
            ++out;
            q += 2;
            continue;
          }
        }
        if (c == quote) {
          if (q + 1 < end && w.at(q + 1) == quote) {          // doubled quote
            buf[out] = (uint8_t)quote;
            rewrite = true;
            ++out;
            q += 2;
            continue;
          }
          break;                                               // closing quote
        }
        if (rewrite) buf[out] = (uint8_t)c;
        ++out;
        ++q;
      }
      if (rewrite) w.wb = -64;                                 // our own stores invalidate the window
      starts[o] = f;
      lens[o] = (int32_t)(out - f);
      valid[o] = 1;
      // skip to the delimiter after the closing quote
      while (q < end && w.at(q) != delim) ++q;
      more = q < end;
      p = q + 1;
    } else {
      int64_t q = p;
      while (q < end && w.at(q) != delim) ++q;
      starts[o] = p;
      lens[o] = (int32_t)(q - p);
      valid[o] = q > p ? 1 : 0;
      more = q < end;
      p = q + 1;
    }
  }
}

}  // namespace

// offs: [nlines + 1] line starts (line i = [offs[i], offs[i+1]), its newline included).  Outputs are column-major:
// starts / lens / valid [ncols][nlines]; row_ok[nlines] = 0 for lines holding only line terminators.
DXA_API int dxa_csv_tokenize(uint8_t* buf, const int64_t* offs, int64_t nlines, int32_t ncols, int32_t delim,
                             int32_t quote, int32_t escape, int64_t* starts, int32_t* lens, uint8_t* valid,
                             uint8_t* row_ok, void* stream) {
  if (nlines <= 0 || ncols <= 0) return 0;
  hipLaunchKernelGGL(csv_tokenize_kernel, dim3((unsigned)((nlines + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     buf, offs, nlines, ncols, (uint32_t)delim & 0xff, (uint32_t)quote & 0xff, (uint32_t)escape & 0xff,
                     starts, lens, valid, row_ok);
  return (int)hipGetLastError();
}
