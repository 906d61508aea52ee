// In-tree LZO1X encoder/decoder (host). Replaces the reference's dlopen of liblzo2
// (src/Merger/LzoDecompressor.cc:35-149, default LZO1X). The decoder accepts the LZO1X bitstream
// that lzo1x_decompress_safe reads: literal runs, M1..M4 matches with the 2-bit trailing-literal
// state, and the M4 end-of-stream marker (0x11 0x00 0x00). Every read and write is bounds checked.
// The encoder is a greedy single-probe hash compressor emitting M2/M3/M4 matches (lzo1x-1 style).
#include <cstring>

#include "uda/codec.h"

namespace uda {

namespace {
constexpr size_t kM2MaxOffset = 0x0800;
constexpr size_t kM3MaxOffset = 0x4000;
constexpr size_t kM4MaxOffset = 0xbfff;
constexpr size_t kM2MaxLen = 8;
constexpr size_t kM3MaxLen = 33;
constexpr size_t kM4MaxLen = 9;
constexpr uint8_t kM3Marker = 32;
constexpr uint8_t kM4Marker = 16;

inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

uint8_t* emit_literals(uint8_t* op, uint8_t* out, const uint8_t* lit, size_t t) {
  if (t == 0) return op;
  if (op == out && t <= 238) {
    *op++ = (uint8_t)(t + 17);
  } else if (t <= 3) {
    op[-2] |= (uint8_t)t;  // trailing-literal state of the previous match
  } else if (t <= 18) {
    *op++ = (uint8_t)(t - 3);
  } else {
    size_t tt = t - 18;
    *op++ = 0;
    while (tt > 255) {
      tt -= 255;
      *op++ = 0;
    }
    *op++ = (uint8_t)tt;
  }
  std::memcpy(op, lit, t);
  return op + t;
}

uint8_t* emit_match(uint8_t* op, size_t m_off, size_t m_len) {
  if (m_len <= kM2MaxLen && m_off <= kM2MaxOffset) {
    m_off -= 1;
    *op++ = (uint8_t)(((m_len - 1) << 5) | ((m_off & 7) << 2));
    *op++ = (uint8_t)(m_off >> 3);
  } else if (m_off <= kM3MaxOffset) {
    m_off -= 1;
    if (m_len <= kM3MaxLen) {
      *op++ = (uint8_t)(kM3Marker | (m_len - 2));
    } else {
      m_len -= kM3MaxLen;
      *op++ = kM3Marker;
      while (m_len > 255) {
        m_len -= 255;
        *op++ = 0;
      }
      *op++ = (uint8_t)m_len;
    }
    *op++ = (uint8_t)(m_off << 2);
    *op++ = (uint8_t)(m_off >> 6);
  } else {
    m_off -= 0x4000;
    if (m_len <= kM4MaxLen) {
      *op++ = (uint8_t)(kM4Marker | ((m_off >> 11) & 8) | (m_len - 2));
    } else {
      m_len -= kM4MaxLen;
      *op++ = (uint8_t)(kM4Marker | ((m_off >> 11) & 8));
      while (m_len > 255) {
        m_len -= 255;
        *op++ = 0;
      }
      *op++ = (uint8_t)m_len;
    }
    *op++ = (uint8_t)(m_off << 2);
    *op++ = (uint8_t)(m_off >> 6);
  }
  return op;
}
}  // namespace

size_t lzo1x_max_compressed_length(size_t n) { return n + n / 16 + 64 + 3; }

size_t lzo1x_compress(const uint8_t* src, size_t n, uint8_t* dst) {
  uint8_t* op = dst;
  constexpr int kBits = 14;
  static thread_local uint32_t table[1 << kBits];
  std::memset(table, 0xFF, sizeof(table));
  size_t ip = 0, lit = 0;
  while (n >= 4 && ip + 4 <= n) {
    const uint32_t h = (load32(src + ip) * 0x1e35a7bdu) >> (32 - kBits);
    const uint32_t cand = table[h];
    table[h] = (uint32_t)ip;
    if (cand != 0xFFFFFFFFu && cand < ip && ip - cand <= kM4MaxOffset && load32(src + cand) == load32(src + ip)) {
      size_t len = 4;
      while (ip + len < n && src[cand + len] == src[ip + len]) ++len;
      op = emit_literals(op, dst, src + lit, ip - lit);
      op = emit_match(op, ip - cand, len);
      ip += len;
      lit = ip;
    } else {
      ++ip;
    }
  }
  op = emit_literals(op, dst, src + lit, n - lit);
  *op++ = kM4Marker | 1;  // end of stream
  *op++ = 0;
  *op++ = 0;
  return (size_t)(op - dst);
}

bool lzo1x_decompress(const uint8_t* in, size_t in_len, uint8_t* out, size_t cap, size_t* out_len) {
  const uint8_t* ip = in;
  const uint8_t* const ip_end = in + in_len;
  uint8_t* op = out;
  uint8_t* const op_end = out + cap;
  size_t t = 0, next = 0, state = 0;
  const uint8_t* m_pos = nullptr;
#define NEED_IP(x) \
  if ((size_t)(ip_end - ip) < (size_t)(x)) return false
#define NEED_OP(x) \
  if ((size_t)(op_end - op) < (size_t)(x)) return false
#define TEST_LB(m) \
  if ((m) < out || (m) >= op) return false
  NEED_IP(1);
  if (*ip > 17) {
    t = (size_t)(*ip++ - 17);
    if (t < 4) {
      next = t;
      goto match_next;
    }
    goto copy_literal_run;
  }
  for (;;) {
    NEED_IP(1);
    t = *ip++;
    if (t < 16) {
      if (state == 0) {
        if (t == 0) {
          while (true) {
            NEED_IP(1);
            if (*ip != 0) break;
            t += 255;
            ++ip;
          }
          t += 15 + *ip++;
        }
        t += 3;
      copy_literal_run:
        NEED_IP(t + 3);  // a literal run is always followed by >= 3 more bytes
        NEED_OP(t);
        std::memcpy(op, ip, t);
        op += t;
        ip += t;
        state = 4;
        continue;
      } else if (state != 4) {  // M1: 2-byte match after 1..3 trailing literals
        next = t & 3;
        NEED_IP(1);
        m_pos = op - 1 - (t >> 2) - ((size_t)*ip++ << 2);
        TEST_LB(m_pos);
        NEED_OP(2);
        op[0] = m_pos[0];
        op[1] = m_pos[1];
        op += 2;
        goto match_next;
      } else {  // M1 after a literal run: 3 bytes, offset 2049..3072
        next = t & 3;
        NEED_IP(1);
        m_pos = op - (1 + kM2MaxOffset) - (t >> 2) - ((size_t)*ip++ << 2);
        t = 3;
      }
    } else if (t >= 64) {  // M2
      next = t & 3;
      NEED_IP(1);
      m_pos = op - 1 - ((t >> 2) & 7) - ((size_t)*ip++ << 3);
      t = (t >> 5) - 1 + 2;
    } else if (t >= 32) {  // M3
      t = (t & 31) + 2;
      if (t == 2) {
        while (true) {
          NEED_IP(1);
          if (*ip != 0) break;
          t += 255;
          ++ip;
        }
        t += 31 + *ip++;
      }
      NEED_IP(2);
      next = (size_t)ip[0] | ((size_t)ip[1] << 8);
      ip += 2;
      m_pos = op - 1 - (next >> 2);
      next &= 3;
    } else {  // M4 (16..31), or end of stream
      m_pos = op - ((t & 8) << 11);
      t = (t & 7) + 2;
      if (t == 2) {
        while (true) {
          NEED_IP(1);
          if (*ip != 0) break;
          t += 255;
          ++ip;
        }
        t += 7 + *ip++;
      }
      NEED_IP(2);
      next = (size_t)ip[0] | ((size_t)ip[1] << 8);
      ip += 2;
      m_pos -= next >> 2;
      next &= 3;
      if (m_pos == op) goto eof_found;
      m_pos -= 0x4000;
    }
    TEST_LB(m_pos);
    NEED_OP(t);
    for (size_t i = 0; i < t; ++i) op[i] = m_pos[i];  // overlapping copy
    op += t;
  match_next:
    state = next;
    t = next;
    NEED_IP(t + 3);
    NEED_OP(t);
    for (size_t i = 0; i < t; ++i) *op++ = *ip++;
  }
eof_found:
  *out_len = (size_t)(op - out);
  return t == 3 && ip == ip_end;
#undef NEED_IP
#undef NEED_OP
#undef TEST_LB
}

}  // namespace uda
