// Order-independent stream checksums: the sum (mod 2^64) of a 64-bit hash of every serialized
// record. The same functions run in the device kernels (generation, validation) and on the host
// (tools/regression.py, StreamValidator), so a checksum computed on one side can be compared with
// the other.
#pragma once
#include <cstdint>

#include "uda/vint.h"  // UDA_HD

namespace uda {

UDA_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// Hash of one serialized record (VInt headers + key + value), consumed as little-endian 8-byte
// words (the last one zero padded). Independent of alignment.
UDA_HD uint64_t record_hash(const uint8_t* p, int64_t len) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)len;
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = 0;
    for (int b = 7; b >= 0; --b) w = (w << 8) | p[i + b];
    h = mix64(h ^ w);
  }
  if (i < len) {
    uint64_t w = 0;
    for (int64_t b = len - 1; b >= i; --b) w = (w << 8) | p[b];
    h = mix64(h ^ w);
  }
  return h;
}

}  // namespace uda
