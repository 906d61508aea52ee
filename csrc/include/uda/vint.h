// Hadoop WritableUtils zero-compressed VInt/VLong codec, usable from host and device code.
//
// Parity: StreamUtility::serializeLong / deserializeLong / getVIntSize / decodeVIntSize
// (src/CommUtils/IOUtility.cc:167-196, 287-333, 367-396). Encoding: values in [-112, 127] take
// one byte; otherwise a length byte (-113..-120 positive, -121..-128 negative) followed by the
// big-endian magnitude bytes, negatives bit-inverted.
#pragma once
#include <cstddef>
#include <cstdint>

#if defined(__HIP__)  // clang HIP language mode (.hip translation units)
#define UDA_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define UDA_HD inline
#endif

namespace uda {

// Number of bytes the encoding of `v` occupies (1..9).
UDA_HD int vint_size(int64_t v) {
  if (v >= -112 && v <= 127) return 1;
  if (v < 0) v ^= -1ll;
  int bits = 0;
  for (uint64_t t = (uint64_t)v; t != 0; t >>= 1) ++bits;
  return (bits + 7) / 8 + 1;
}

// Total encoded size given only the first byte (as a signed byte value).
UDA_HD int vint_decode_size(int first) {
  if (first >= -112) return 1;
  if (first < -120) return -119 - first;
  return -111 - first;
}

// Encode into `out` (must hold 9 bytes). Returns bytes written.
UDA_HD int vint_encode(int64_t v, uint8_t* out) {
  if (v >= -112 && v <= 127) {
    out[0] = (uint8_t)(int8_t)v;
    return 1;
  }
  int len = -112;
  if (v < 0) {
    v ^= -1ll;
    len = -120;
  }
  for (uint64_t t = (uint64_t)v; t != 0; t >>= 8) --len;
  out[0] = (uint8_t)(int8_t)len;
  int n = (len < -120) ? -(len + 120) : -(len + 112);
  for (int i = 0; i < n; ++i) out[1 + i] = (uint8_t)(((uint64_t)v >> ((n - 1 - i) * 8)) & 0xFF);
  return n + 1;
}

// Decode from [p, p+avail). Returns bytes consumed, or 0 if the encoding is truncated.
UDA_HD int vint_decode(const uint8_t* p, size_t avail, int64_t* out) {
  if (avail < 1) return 0;
  int8_t b = (int8_t)p[0];
  if (b >= -112) {
    *out = b;
    return 1;
  }
  bool neg = b < -120;
  int n = neg ? (-120 - b) : (-112 - b);
  if ((size_t)(n + 1) > avail) return 0;
  int64_t t = 0;
  for (int i = 0; i < n; ++i) t = (t << 8) | p[1 + i];
  if (neg) t ^= -1ll;
  *out = t;
  return n + 1;
}

// IFile end-of-stream marker: VInt(-1) VInt(-1) (src/Merger/StreamRW.cc:205-221).
constexpr int32_t kEofMarker = -1;
constexpr int kEofBytes = 2;

}  // namespace uda
