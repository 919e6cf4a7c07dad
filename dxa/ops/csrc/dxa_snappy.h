// Snappy (host side): the raw block format and the xerial snappy-java stream framing Kafka uses for compression
// codec 2.
//   Raw block: varint uncompressed length | elements, each a tag byte whose low 2 bits pick the kind:
//     00 literal  — length-1 in the upper 6 bits (< 60), or 60..63: 1..4 little-endian length-1 bytes follow;
//     01 copy     — length 4..11 in bits 2..4, offset bits 8..10 in bits 5..7, offset low byte follows;
//     10 copy     — length 1..64 in the upper 6 bits, 16-bit little-endian offset follows;
//     11 copy     — length 1..64, 32-bit little-endian offset follows.
//   xerial stream (SnappyOutputStream, what the Java producer writes): magic 82 'SNAPPY' 00 | version i32 BE |
//     compatible version i32 BE | chunks of (i32 BE compressed length | raw block), one per 32 KiB of input.
//   A consumer also accepts a bare raw block (librdkafka producers before the framing, SnappyInputStream's
//   fallback).  The device decoder (snappy.hip) reads the same raw blocks.
#pragma once
#include <cstdint>

namespace dxa {
namespace snappy {

int64_t max_compressed_length(int64_t n);
// Compress one raw block (any size; matched in 64 KiB fragments like the reference compressor).
int64_t compress_raw(const uint8_t* src, int64_t n, uint8_t* dst);
// Uncompressed length from the varint preamble (-1 malformed); *hdr = preamble bytes.
int64_t raw_length(const uint8_t* src, int64_t n, int32_t* hdr);
// Decompress one raw block into dst[cap]; returns the size or -1.
int64_t decompress_raw(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);

bool is_xerial(const uint8_t* src, int64_t n);
// xerial framing: bound, compress (32 KiB chunks), and walk the chunk table (counts when the arrays are null;
// returns the chunk count or -1 malformed).  Offsets are relative to src.
int64_t xerial_bound(int64_t n);
int64_t xerial_compress(const uint8_t* src, int64_t n, uint8_t* dst);
int64_t xerial_chunks(const uint8_t* src, int64_t n, int64_t* off, int32_t* len, int64_t* out_len, int64_t max);
// Whole Kafka snappy payload (xerial stream or one raw block) → dst[cap]; returns the size or -1.
int64_t decompress_payload(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
int64_t payload_length(const uint8_t* src, int64_t n);

}  // namespace snappy
}  // namespace dxa
