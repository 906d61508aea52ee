// Device comparison of generic keys (any Hadoop key class after key_content_offset): the total
// order of the generic merge is (content bytes lexicographically, content length, record ordinal).
// Elem.hi holds the first 8 content bytes big-endian, Elem.lo = (min(len, 0xFFFF) << 48) | ordinal.
#pragma once
#include "kernels.h"

namespace uda {
namespace gpu {

constexpr uint64_t kGenOrdMask = 0xFFFFFFFFFFFFull;

// Big-endian 8 bytes of p (zero padded past n bytes).
__device__ __forceinline__ uint64_t load_be8(const uint8_t* p, int n) {
  uint64_t v = 0;
  if (n >= 8) {
    uint64_t w;
    __builtin_memcpy(&w, p, 8);
    return __builtin_bswap64(w);
  }
  for (int i = 0; i < 8; ++i) v = (v << 8) | (uint64_t)(i < n ? p[i] : 0);
  return v;
}

// a <= b in the total order; prefix ties between keys longer than 8 bytes are settled on the raw
// key bytes, read through the per-record side tables 8 bytes at a time.
__device__ __forceinline__ bool generic_le(const GenericKeyCtx& ctx, const Elem& a, const Elem& b) {
  if (a.hi != b.hi) return a.hi < b.hi;
  if ((a.lo >> 48) > 8 && (b.lo >> 48) > 8) {
    const uint64_t ga = a.lo & kGenOrdMask, gb = b.lo & kGenOrdMask;
    const uint8_t* pa = ctx.keyptr[ga];
    const uint8_t* pb = ctx.keyptr[gb];
    const int la = ctx.keylen[ga], lb = ctx.keylen[gb];
    const int n = la < lb ? la : lb;
    for (int i = 8; i < n; i += 8) {
      const uint64_t x = load_be8(pa + i, n - i), y = load_be8(pb + i, n - i);
      if (x != y) return x < y;
    }
    if (la != lb) return la < lb;
  }
  return a.lo <= b.lo;
}

// Length of the common prefix of two keys, at most `limit`.
__device__ __forceinline__ int key_lcp(const uint8_t* a, int la, const uint8_t* b, int lb, int limit) {
  const int n = min(min(la, lb), limit);
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x, y;
    __builtin_memcpy(&x, a + i, 8);
    __builtin_memcpy(&y, b + i, 8);
    if (x != y) return i + (__builtin_ctzll(x ^ y) >> 3);  // little-endian: first differing byte
  }
  while (i < n && a[i] == b[i]) ++i;
  return i;
}

}  // namespace gpu
}  // namespace uda
