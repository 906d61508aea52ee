// Hadoop block-stream framing and codec selection. See uda/codec.h.
#include <algorithm>
#include <cstring>

#include "uda/codec.h"
#include "uda/error.h"

namespace uda {

Codec codec_from_class(const std::string& cls, bool* unsupported) {
  *unsupported = false;
  if (cls.empty() || cls == "null") return Codec::kNone;
  if (cls.find("SnappyCodec") != std::string::npos) return Codec::kSnappy;
  if (cls.find("LzoCodec") != std::string::npos || cls.find("LzopCodec") != std::string::npos) return Codec::kLzo;
  *unsupported = true;  // getCompAlg (reducer.cc:439-450) throws on anything else
  return Codec::kNone;
}

const char* codec_name(Codec c) {
  switch (c) {
    case Codec::kSnappy: return "snappy";
    case Codec::kLzo: return "lzo1x";
    default: return "none";
  }
}

namespace {
void put_be32(std::vector<uint8_t>* v, uint32_t x) {
  v->push_back((uint8_t)(x >> 24));
  v->push_back((uint8_t)(x >> 16));
  v->push_back((uint8_t)(x >> 8));
  v->push_back((uint8_t)x);
}
uint32_t get_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
}  // namespace

std::vector<uint8_t> block_compress(Codec c, const uint8_t* src, size_t n, size_t block_size) {
  std::vector<uint8_t> out;
  if (block_size == 0) block_size = 256 * 1024;
  std::vector<uint8_t> tmp;
  for (size_t off = 0; off < n; off += block_size) {
    const size_t len = std::min(block_size, n - off);
    put_be32(&out, (uint32_t)len);
    size_t clen = 0;
    if (c == Codec::kSnappy) {
      tmp.resize(snappy_max_compressed_length(len));
      clen = snappy_compress(src + off, len, tmp.data());
    } else if (c == Codec::kLzo) {
      tmp.resize(lzo1x_max_compressed_length(len));
      clen = lzo1x_compress(src + off, len, tmp.data());
    } else {
      throw UdaError("block_compress: no codec");
    }
    put_be32(&out, (uint32_t)clen);
    out.insert(out.end(), tmp.begin(), tmp.begin() + (long)clen);
  }
  return out;
}

void BlockDecoder::feed(const uint8_t* p, size_t n) {
  if (in_pos_ > 0 && in_pos_ == in_.size()) {
    in_.clear();
    in_pos_ = 0;
  } else if (in_pos_ > (1u << 20) && in_pos_ > in_.size() / 2) {
    in_.erase(in_.begin(), in_.begin() + (long)in_pos_);
    in_pos_ = 0;
  }
  in_.insert(in_.end(), p, p + n);
}

bool BlockDecoder::decode_some() {
  const size_t avail = in_.size() - in_pos_;
  if (block_remaining_ == 0) {
    if (avail < 4) return false;
    block_remaining_ = get_be32(in_.data() + in_pos_);
    in_pos_ += 4;
    ++blocks_;
    return true;  // a zero-length block is legal; loop again
  }
  if (avail < 4) return false;
  const uint32_t clen = get_be32(in_.data() + in_pos_);
  if (avail < 4 + (size_t)clen) return false;
  const uint8_t* src = in_.data() + in_pos_ + 4;
  if (out_pos_ == out_.size()) {
    out_.clear();
    out_pos_ = 0;
  }
  const size_t base = out_.size();
  out_.resize(base + (size_t)block_remaining_);
  size_t got = 0;
  bool ok = (codec_ == Codec::kSnappy)
                ? snappy_decompress(src, clen, out_.data() + base, (size_t)block_remaining_, &got)
                : lzo1x_decompress(src, clen, out_.data() + base, (size_t)block_remaining_, &got);
  if (!ok) throw UdaError(std::string("corrupt ") + codec_name(codec_) + " block");
  out_.resize(base + got);
  block_remaining_ -= (int64_t)got;
  in_pos_ += 4 + (size_t)clen;
  return true;
}

size_t BlockDecoder::read(uint8_t* dst, size_t cap) {
  while (out_pos_ == out_.size()) {
    if (!decode_some()) return 0;
  }
  const size_t n = std::min(cap, out_.size() - out_pos_);
  std::memcpy(dst, out_.data() + out_pos_, n);
  out_pos_ += n;
  return n;
}

}  // namespace uda
