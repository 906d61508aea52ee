// Key comparator family and key normalization (host + device).
//
// Parity: src/Merger/CompareFunc.cc:29-113. The Java key class name selects one of three raw
// comparators over the *serialized* key bytes:
//   Text                               -> skip the VInt length prefix, memcmp, then length
//   Boolean/Byte/Short/Int/LongWritable-> memcmp of the raw bytes, then length
//   BytesWritable/ImmutableBytesWritable -> skip the 4-byte length, memcmp, then length
// Anything else is unsupported (the reference throws -> host falls back to vanilla shuffle).
//
// MI355X design: instead of calling the comparator O(log K) times per record from a heap, the GPU
// path normalizes every key once into a fixed-width big-endian prefix (`KeyNorm`) so almost all
// comparisons are two 64-bit integer compares; only prefix ties on keys longer than the prefix
// fall back to `key_compare` on the raw bytes.
#pragma once
#include <cstdint>
#include <cstring>

#include "uda/vint.h"

namespace uda {

enum class KeyKind : int { kText = 0, kRaw = 1, kBytes = 2, kUnsupported = -1 };

// Map a Java key class name to a comparator kind (CompareFunc.cc:95-113).
KeyKind key_kind_from_class(const char* java_class_name);
const char* key_kind_name(KeyKind k);

constexpr int kBytesWritableLenBytes = 4;  // LENGTH_BYTES in the reference

// Offset of the comparable content inside the serialized key.
UDA_HD int key_content_offset(KeyKind kind, const uint8_t* key, int len) {
  if (kind == KeyKind::kText) {
    if (len <= 0) return 0;
    int s = vint_decode_size((int)(int8_t)key[0]);
    return s > len ? len : s;
  }
  if (kind == KeyKind::kBytes) return len < kBytesWritableLenBytes ? len : kBytesWritableLenBytes;
  return 0;
}

UDA_HD int bytes_compare(const uint8_t* a, int la, const uint8_t* b, int lb) {
  int n = la < lb ? la : lb;
  for (int i = 0; i < n; ++i) {
    if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  }
  return la - lb;
}

// Full comparator on serialized keys. Sign matches the reference comparator.
UDA_HD int key_compare(KeyKind kind, const uint8_t* a, int la, const uint8_t* b, int lb) {
  int oa = key_content_offset(kind, a, la);
  int ob = key_content_offset(kind, b, lb);
  return bytes_compare(a + oa, la - oa, b + ob, lb - ob);
}

// Big-endian load of up to 8 bytes, zero padded on the right.
UDA_HD uint64_t load_be_prefix(const uint8_t* p, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | (uint64_t)(i < n ? p[i] : 0);
  return v;
#else
  // host: one unaligned load (or a short copy into a zeroed word) and a byte swap
  uint64_t w = 0;
  if (n >= 8)
    __builtin_memcpy(&w, p, 8);
  else if (n > 0)
    __builtin_memcpy(&w, p, (size_t)n);
  return __builtin_bswap64(w);
#endif
}

// Normalized key: the first 16 content bytes (big-endian, zero padded) and the content length.
// Order on (k0, k1) is consistent with memcmp on the content; when both contents are <= 16 bytes
// and (k0, k1) tie, the shorter content is smaller (the reference's `len1 - len2` tie-break).
struct KeyNorm {
  uint64_t k0;
  uint64_t k1;
  uint32_t len;  // content length (after skipping the VInt / 4-byte prefix)
  uint32_t off;  // content offset inside the serialized key
};

UDA_HD KeyNorm key_normalize(KeyKind kind, const uint8_t* key, int len) {
  KeyNorm n;
  int o = key_content_offset(kind, key, len);
  int cl = len - o;
  n.k0 = load_be_prefix(key + o, cl);
  n.k1 = load_be_prefix(key + o + (cl > 8 ? 8 : cl), cl > 8 ? cl - 8 : 0);
  n.len = (uint32_t)cl;
  n.off = (uint32_t)o;
  return n;
}

// Compare two normalized keys. Returns <0, 0, >0; `needs_full` is set when the prefixes tie and
// at least one content is longer than 16 bytes (the caller must then run key_compare).
UDA_HD int keynorm_compare(const KeyNorm& a, const KeyNorm& b, bool* needs_full) {
  *needs_full = false;
  if (a.k0 != b.k0) return a.k0 < b.k0 ? -1 : 1;
  if (a.k1 != b.k1) return a.k1 < b.k1 ? -1 : 1;
  if (a.len <= 16 && b.len <= 16) return (int)a.len - (int)b.len;
  *needs_full = true;
  return 0;
}

}  // namespace uda
