// LZ4 block + frame codec (host side).  Block format: sequences of
//   token (hi nibble literal length, lo nibble match length - 4; 15 = "more bytes follow", each 255 adds and a
//   byte < 255 ends) | literals | offset u16 LE | match length extension
// with the last 5 bytes always literals and no match starting in the last 12 bytes.  Frame format (v1.6): magic
// 0x184D2204 | FLG | BD | [content size u64] | HC | blocks (u32 LE size, bit 31 = stored uncompressed) | u32 0.
// The device decoder (lz4.hip) reads the same frames; Kafka uses the frame format for compression codec 3.
#pragma once
#include <cstdint>

namespace dxa {
namespace lz4 {

int64_t block_bound(int64_t n);
// Compress one independent block; returns the compressed size (<= block_bound(n)).
int64_t compress_block(const uint8_t* src, int64_t n, uint8_t* dst);
// Decompress one block into dst[cap]; returns the decompressed size or -1 on malformed input / overflow.
int64_t decompress_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
uint32_t xxh32(const uint8_t* p, int64_t n, uint32_t seed);
// High-compression block (hash chains, `depth` candidates per position, lazy matching); same format.
int64_t compress_block_hc(const uint8_t* src, int64_t n, uint8_t* dst, int depth);
// Frame: compress with independent blocks of `block_size` (<= 4 MiB) bytes using `threads` workers.  `level`
// <= 2 is the greedy compressor; L >= 3 is the high-compression mode searching 2^(L-1) candidates (max 4096).
int64_t frame_bound(int64_t n, int32_t block_size);
int64_t compress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int32_t block_size, int32_t threads,
                       int32_t level = 0);
// Walk a frame's block table.  Fills up to max_blocks entries (may be null to count); returns the block count, or
// -1 malformed / -2 unsupported (dependent blocks, dictionary).  content_size = -1 when the frame omits it.
int64_t frame_blocks(const uint8_t* src, int64_t n, int64_t* comp_off, int32_t* comp_len, uint8_t* stored,
                     int64_t max_blocks, int64_t* content_size, int32_t* max_block_size, int64_t* frame_end);
// Decompress a whole frame (or several concatenated frames); returns the size or a negative error.
int64_t decompress_frame(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);

}  // namespace lz4
}  // namespace dxa
