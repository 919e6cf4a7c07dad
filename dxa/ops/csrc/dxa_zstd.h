// Zstandard (RFC 8878) on the host: the reference decoder of the Kafka codec-4 ingest path (CPU runs, tests) and
// the frame walker the device planner uses.  The device decoder is zstd.hip (one wave per frame).
//   Frame: magic FD2FB528 | header descriptor | [window descriptor] | [dictionary id] | [content size] | blocks
//          (3-byte header: last flag, type raw / RLE / compressed, size) | [xxhash64 checksum, 4 bytes]
//   Compressed block: literals section (raw / RLE / Huffman-coded in 1 or 4 streams / treeless = previous table)
//          | sequences section (count, modes, FSE tables for literal lengths, offsets, match lengths — predefined,
//          RLE, described, or repeated — then one backward bitstream of interleaved states).
// Skippable frames (184D2A5x) are skipped.  Dictionaries are not supported (Kafka never sets one).
#pragma once
#include <cstdint>

namespace dxa {
namespace zstd {

// Frame facts from its header and block headers (no entropy decoding): frame end offset, a decompressed-size bound
// (content size when the header has it, else blocks x block maximum), the window size, whether it carries a
// checksum.  Returns 0, or -1 malformed / -2 dictionary / -3 not a zstd frame.
struct FrameInfo {
  int64_t header_len;
  int64_t end;                 // offset just past the frame (checksum included)
  int64_t content_size;        // -1 when absent
  int64_t bound;               // decompressed size upper bound
  int64_t window;
  int32_t nblocks;
  int32_t checksum;
};
int frame_info(const uint8_t* src, int64_t n, FrameInfo* fi);

// Decompress one frame (or several concatenated, skippable ones skipped) into dst[cap]; returns the size or a
// negative error code (see zstd.cpp kErr*).
int64_t decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
// Sum of the bounds of every frame in src (-1 malformed).
int64_t decompressed_bound(const uint8_t* src, int64_t n);

}  // namespace zstd
}  // namespace dxa
