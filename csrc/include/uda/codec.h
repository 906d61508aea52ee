// Map-output compression codecs and Hadoop block-stream framing.
//
// Parity: DecompressorWrapper + LzoDecompressor + SnappyDecompressor (src/Merger/
// DecompressorWrapper.cc, LzoDecompressor.cc, SnappyDecompressor.cc). The reference dlopens
// liblzo2 / libsnappy; neither exists here, so both decoders are implemented in-tree (host C++;
// the GPU engine has its own per-block device decoders). Framing (Hadoop BlockCompressorStream):
//   block := [u32 BE uncompressed_len] { [u32 BE compressed_len][compressed bytes] }+
// The reference assumes one compressed chunk per block (LzoDecompressor.cc:151-167); we accept
// several chunks per block, which Hadoop emits when a block's compressed output is split.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace uda {

enum class Codec { kNone = 0, kSnappy = 1, kLzo = 2 };

// Map a Hadoop codec class name ("...SnappyCodec", "...LzoCodec") to a codec; kNone for ""/null.
// Unsupported names return kNone and set *unsupported.
Codec codec_from_class(const std::string& cls, bool* unsupported);
const char* codec_name(Codec c);

// ---- Snappy (raw format: varint uncompressed length, then literal/copy tags)
size_t snappy_max_compressed_length(size_t n);
size_t snappy_compress(const uint8_t* src, size_t n, uint8_t* dst);
bool snappy_uncompressed_length(const uint8_t* src, size_t n, size_t* out);
bool snappy_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

// ---- LZO1X (the format liblzo2's lzo1x_decompress_safe reads)
size_t lzo1x_max_compressed_length(size_t n);
size_t lzo1x_compress(const uint8_t* src, size_t n, uint8_t* dst);
bool lzo1x_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len);

// Compress `n` bytes into Hadoop block framing with blocks of at most `block_size` raw bytes.
std::vector<uint8_t> block_compress(Codec c, const uint8_t* src, size_t n, size_t block_size);

// Incremental decoder of a framed stream: feed compressed bytes in arbitrary pieces, read raw.
class BlockDecoder {
 public:
  explicit BlockDecoder(Codec c) : codec_(c) {}
  // Append compressed input.
  void feed(const uint8_t* p, size_t n);
  // Copy up to `cap` decoded bytes into dst; returns bytes produced (0 = need more input).
  // Throws UdaError on a corrupt stream.
  size_t read(uint8_t* dst, size_t cap);
  // True when no buffered raw bytes remain and the input ended on a block boundary.
  bool idle() const { return out_pos_ == out_.size() && in_.size() == in_pos_ && block_remaining_ == 0; }
  int64_t blocks() const { return blocks_; }

 private:
  bool decode_some();
  Codec codec_;
  std::vector<uint8_t> in_;
  size_t in_pos_ = 0;
  std::vector<uint8_t> out_;
  size_t out_pos_ = 0;
  int64_t block_remaining_ = 0;  // raw bytes of the current block not yet produced
  int64_t blocks_ = 0;
};

}  // namespace uda
