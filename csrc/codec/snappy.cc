// In-tree Snappy (raw format) encoder/decoder (host). Replaces the reference's dlopen of
// libsnappy (src/Merger/SnappyDecompressor.cc:47-87). Format: varint uncompressed length, then
// elements whose tag's low two bits select literal (00), copy with 1-byte offset (01), 2-byte
// offset (10) or 4-byte offset (11).
#include <cstring>

#include "uda/codec.h"

namespace uda {

namespace {
inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

uint8_t* emit_literal(uint8_t* op, const uint8_t* lit, size_t len) {
  size_t n = len - 1;
  if (n < 60) {
    *op++ = (uint8_t)(n << 2);
  } else {
    int bytes = n < (1u << 8) ? 1 : n < (1u << 16) ? 2 : n < (1u << 24) ? 3 : 4;
    *op++ = (uint8_t)((59 + bytes) << 2);
    for (int i = 0; i < bytes; ++i) *op++ = (uint8_t)(n >> (8 * i));
  }
  std::memcpy(op, lit, len);
  return op + len;
}

uint8_t* emit_copy_upto64(uint8_t* op, size_t offset, size_t len) {
  if (len >= 4 && len < 12 && offset < 2048) {
    *op++ = (uint8_t)(1 | ((len - 4) << 2) | ((offset >> 8) << 5));
    *op++ = (uint8_t)(offset & 0xFF);
  } else if (offset < 65536) {
    *op++ = (uint8_t)(2 | ((len - 1) << 2));
    *op++ = (uint8_t)(offset & 0xFF);
    *op++ = (uint8_t)(offset >> 8);
  } else {
    *op++ = (uint8_t)(3 | ((len - 1) << 2));
    for (int i = 0; i < 4; ++i) *op++ = (uint8_t)(offset >> (8 * i));
  }
  return op;
}

uint8_t* emit_copy(uint8_t* op, size_t offset, size_t len) {
  while (len >= 68) {
    op = emit_copy_upto64(op, offset, 64);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_upto64(op, offset, 60);
    len -= 60;
  }
  return emit_copy_upto64(op, offset, len);
}
}  // namespace

size_t snappy_max_compressed_length(size_t n) { return 32 + n + n / 6; }

size_t snappy_compress(const uint8_t* src, size_t n, uint8_t* dst) {
  uint8_t* op = dst;
  // varint length
  size_t v = n;
  while (v >= 0x80) {
    *op++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *op++ = (uint8_t)v;
  if (n == 0) return (size_t)(op - dst);
  constexpr int kBits = 14;
  static thread_local uint32_t table[1 << kBits];
  std::memset(table, 0, sizeof(table));
  size_t ip = 0, lit = 0;
  while (n >= 4 && ip + 4 <= n) {
    const uint32_t h = (load32(src + ip) * 0x1e35a7bdu) >> (32 - kBits);
    const size_t cand = table[h];
    table[h] = (uint32_t)ip;
    if (cand < ip && ip - cand <= 0xFFFFFFFFu && load32(src + cand) == load32(src + ip) &&
        (ip - cand) < (1u << 31)) {
      size_t len = 4;
      while (ip + len < n && src[cand + len] == src[ip + len]) ++len;
      if (ip > lit) op = emit_literal(op, src + lit, ip - lit);
      op = emit_copy(op, ip - cand, len);
      ip += len;
      lit = ip;
    } else {
      ++ip;
    }
  }
  if (lit < n) op = emit_literal(op, src + lit, n - lit);
  return (size_t)(op - dst);
}

bool snappy_uncompressed_length(const uint8_t* src, size_t n, size_t* out) {
  size_t v = 0;
  int shift = 0;
  for (size_t i = 0; i < n && i < 10; ++i) {
    v |= (size_t)(src[i] & 0x7F) << shift;
    if (!(src[i] & 0x80)) {
      *out = v;
      return true;
    }
    shift += 7;
  }
  return false;
}

bool snappy_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
  size_t ip = 0, ulen = 0;
  {
    size_t v = 0;
    int shift = 0;
    bool ok = false;
    while (ip < n && ip < 10) {
      uint8_t b = src[ip++];
      v |= (size_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) {
        ok = true;
        break;
      }
      shift += 7;
    }
    if (!ok) return false;
    ulen = v;
  }
  if (ulen > cap) return false;
  size_t op = 0;
  while (ip < n) {
    const uint8_t tag = src[ip++];
    const int type = tag & 3;
    if (type == 0) {
      size_t len = (size_t)(tag >> 2);
      if (len >= 60) {
        const int bytes = (int)len - 59;
        if (ip + (size_t)bytes > n) return false;
        len = 0;
        for (int i = 0; i < bytes; ++i) len |= (size_t)src[ip + i] << (8 * i);
        ip += (size_t)bytes;
      }
      len += 1;
      if (ip + len > n || op + len > ulen) return false;
      std::memcpy(dst + op, src + ip, len);
      ip += len;
      op += len;
    } else {
      size_t len, off;
      if (type == 1) {
        if (ip + 1 > n) return false;
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | src[ip];
        ip += 1;
      } else if (type == 2) {
        if (ip + 2 > n) return false;
        len = 1 + (tag >> 2);
        off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) return false;
        len = 1 + (tag >> 2);
        off = (size_t)load32(src + ip);
        ip += 4;
      }
      if (off == 0 || off > op || op + len > ulen) return false;
      // overlapping copy: byte-wise when the source overlaps the destination
      for (size_t i = 0; i < len; ++i) dst[op + i] = dst[op - off + i];
      op += len;
    }
  }
  if (op != ulen) return false;
  *out_len = op;
  return true;
}

}  // namespace uda
