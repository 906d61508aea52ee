// F6 — block-decompress kernels (Snappy raw format, LZO1X) for Hadoop block-compressed map
// outputs, decoded in HBM so the compressed bytes are what crosses PCIe / the network.
//
// Reference: DecompressorWrapper::doDecompress (src/Merger/DecompressorWrapper.cc:168-197) feeding
// liblzo2 / libsnappy one block at a time on the merge thread. Here every Hadoop block is decoded
// by one wave64, all blocks of all runs in one launch:
//   * the compressed stream of the wave's block is staged through a per-wave LDS window; the tag /
//     opcode parse is wave-uniform (every lane decodes the same element; the values are scalar),
//   * literals and back-references are copied by the 64 lanes cooperatively; an overlapping copy
//     (offset < length) becomes a periodic fill out[op+i] = out[op-off + i % off],
//   * a back-reference that reads bytes this wave stored since the last store fence first waits
//     for its stores (workgroup-scope fence: the wave's own stores are visible through the CU's
//     write-through L1 once they completed).
// Format parity with the host decoders in csrc/codec/{snappy,lzo}.cc (same bounds checks); a
// corrupt block sets its status word and the caller raises.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "kernels.h"

namespace uda {
namespace gpu {

namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kWin = 2048;  // per-wave LDS window of compressed input

struct Wave {
  const uint8_t* in;
  uint8_t* out;
  uint8_t* win;       // LDS window
  int64_t win_base;   // stream offset of win[0]
  int64_t win_end;    // stream offset one past the valid window bytes
  int64_t in_end;     // end of this block's compressed bytes
  int64_t flushed;    // output offset below which every store of this wave has completed
  int64_t clip;       // prefix decode: no byte at or past this output offset is written
  bool prefix;        // a prefix decode (stops at clip); else clip is the block's end
  int lane;
  uint32_t rw;        // register window: this lane's 4 bytes of the 256-byte window at win_base
};

__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

__device__ __forceinline__ int64_t uni(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Register window (R): the 256 compressed bytes at win_base spread 4 per lane over a VGPR; a byte is
// one v_readlane (a few cycles) instead of a dependent LDS read (~100) on the parse's critical path.
// Refilled by one coalesced 256-byte load; lanes past the block end hold zeros.
constexpr int kRegWin = 256;
struct __attribute__((packed, aligned(1))) U32p {
  uint32_t v;
};
template <bool R>
__device__ __forceinline__ bool ensure(Wave& w, int64_t ip, int need) {
  if (ip + need > w.in_end) return false;
  if (ip >= w.win_base && ip + need <= w.win_end) return true;
  if (R) {
    const int64_t base = ip & ~(int64_t)3;
    const int64_t end = min(base + kRegWin, w.in_end);
    const int64_t p = base + 4 * w.lane;
    uint32_t v = 0;
    if (p + 4 <= end) {
      v = reinterpret_cast<const U32p*>(w.in + p)->v;
    } else {
      for (int k = 0; k < 4; ++k)
        if (p + k < end) v |= (uint32_t)w.in[p + k] << (8 * k);
    }
    w.rw = v;
    w.win_base = base;
    w.win_end = end;
    return true;
  }
  wave_sync();
  const int64_t base = ip & ~(int64_t)15;
  const int64_t end = min(base + kWin, w.in_end);
  for (int i = w.lane * 16; i < kWin; i += 64 * 16) {
    const int64_t p = base + i;
    if (p + 16 <= end) {
      // 16-byte aligned vector load when the source alignment allows, bytes otherwise
      if ((((uintptr_t)(w.in + p)) & 15) == 0) {
        *reinterpret_cast<uint4*>(w.win + i) = *reinterpret_cast<const uint4*>(w.in + p);
      } else {
        for (int k = 0; k < 16; ++k) w.win[i + k] = w.in[p + k];
      }
    } else {
      for (int k = 0; k < 16; ++k) w.win[i + k] = (p + k < end) ? w.in[p + k] : 0;
    }
  }
  wave_sync();
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes of every lane done before reads
  wave_sync();
  w.win_base = base;
  w.win_end = end;
  return true;
}

template <bool R>
__device__ __forceinline__ uint32_t byte_at(const Wave& w, int64_t ip) {
  if (R) {
    const int d = (int)(ip - w.win_base);
    const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)w.rw, d >> 2);
    return (word >> (8 * (d & 3))) & 0xFF;
  }
  return (uint32_t)w.win[ip - w.win_base];
}

// 16 bytes per lane at any alignment: gfx950 runs in unaligned-access mode, so a packed 16-byte
// struct compiles to one global_load/store_dwordx4 (1 KiB per wave step instead of 64 bytes).
struct __attribute__((packed, aligned(1))) U128 {
  uint32_t a, b, c, d;
};

// Non-overlapping copy dst[0, len) = src[0, len) by the 64 lanes.
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, int64_t len, int lane) {
  const int64_t nv = len & ~(int64_t)15;
  for (int64_t i = (int64_t)lane * 16; i < nv; i += 64 * 16)
    *reinterpret_cast<U128*>(dst + i) = *reinterpret_cast<const U128*>(src + i);
  for (int64_t i = nv + lane; i < len; i += 64) dst[i] = src[i];
}

__device__ __forceinline__ void copy_literal(Wave& w, int64_t op, int64_t ip, int64_t len) {
  len = min(len, w.clip - op);  // a prefix decode keeps only the bytes below its clip
  if (len > 0) wave_copy(w.out + op, w.in + ip, len, w.lane);
}

// out[op .. op+len) = out[op-off ...] with LZ77 overlap semantics.
__device__ __forceinline__ void copy_match(Wave& w, int64_t op, int64_t off, int64_t len) {
  len = min(len, w.clip - op);  // the source bytes below the clip were all written
  if (len <= 0) return;
  const int64_t src = op - off;
  if (src + min(off, len) > w.flushed) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's stores completed
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    w.flushed = op;
  }
  if (off >= len) {
    wave_copy(w.out + op, w.out + src, len, w.lane);
  } else {
    for (int64_t i = w.lane; i < len; i += 64) w.out[op + i] = w.out[src + (i % off)];
  }
}

template <bool R>
__device__ bool snappy_chunk(Wave& w, int64_t ip, int64_t cend, int64_t op, int64_t oend, int64_t* produced) {
  w.in_end = cend;
  // varint uncompressed length
  int64_t ulen = 0;
  int shift = 0;
  for (;;) {
    if (shift > 35 || !ensure<R>(w, ip, 1)) return false;
    const uint32_t b = byte_at<R>(w, ip++);
    ulen |= (int64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
    shift += 7;
  }
  ulen = uni(ulen);
  if (op + ulen > oend) return false;
  const int64_t op0 = op, uend = op + ulen;
  while (ip < cend) {
    if (w.prefix && op >= w.clip) {  // prefix decode: everything wanted is out
      *produced = ulen;
      return true;
    }
    if (!ensure<R>(w, ip, 1)) return false;
    const uint32_t tag = byte_at<R>(w, ip++);
    const uint32_t type = tag & 3;
    if (type == 0) {
      int64_t len = tag >> 2;
      if (len >= 60) {
        const int nb = (int)len - 59;
        if (!ensure<R>(w, ip, nb)) return false;
        len = 0;
        for (int i = 0; i < nb; ++i) len |= (int64_t)byte_at<R>(w, ip + i) << (8 * i);
        ip += nb;
      }
      len += 1;
      if (ip + len > cend || op + len > uend) return false;
      copy_literal(w, op, ip, len);
      ip += len;
      op += len;
    } else {
      int64_t len, off;
      if (type == 1) {
        if (!ensure<R>(w, ip, 1)) return false;
        len = 4 + ((tag >> 2) & 7);
        off = ((int64_t)(tag >> 5) << 8) | byte_at<R>(w, ip);
        ip += 1;
      } else if (type == 2) {
        if (!ensure<R>(w, ip, 2)) return false;
        len = 1 + (tag >> 2);
        off = (int64_t)byte_at<R>(w, ip) | ((int64_t)byte_at<R>(w, ip + 1) << 8);
        ip += 2;
      } else {
        if (!ensure<R>(w, ip, 4)) return false;
        len = 1 + (tag >> 2);
        off = (int64_t)byte_at<R>(w, ip) | ((int64_t)byte_at<R>(w, ip + 1) << 8) | ((int64_t)byte_at<R>(w, ip + 2) << 16) |
              ((int64_t)byte_at<R>(w, ip + 3) << 24);
        ip += 4;
      }
      if (off == 0 || off > op - op0 || op + len > uend) return false;
      copy_match(w, op, off, len);
      op += len;
    }
  }
  if (op != uend) return false;
  *produced = ulen;
  return true;
}

// LZO1X: the state machine of csrc/codec/lzo.cc, wave-uniform.
template <bool R>
__device__ bool lzo_chunk(Wave& w, int64_t ip, int64_t ip_end, int64_t op, int64_t oend, int64_t* produced) {
  w.in_end = ip_end;
  const int64_t out0 = op;
  int64_t t = 0, next = 0, state = 0, m_pos = 0;
  bool lit_first = false;
  if (!ensure<R>(w, ip, 1)) return false;
  if (byte_at<R>(w, ip) > 17) {
    t = (int64_t)byte_at<R>(w, ip) - 17;
    ++ip;
    if (t < 4) {
      next = t;
      goto match_next;
    }
    lit_first = true;
  }
  for (;;) {
    if (w.prefix && op >= w.clip) {  // prefix decode: everything wanted is out
      *produced = oend - out0;
      return true;
    }
    if (lit_first) {
      lit_first = false;
      goto copy_literal_run;
    }
    if (!ensure<R>(w, ip, 1)) return false;
    t = byte_at<R>(w, ip++);
    if (t < 16) {
      if (state == 0) {
        if (t == 0) {
          for (;;) {
            if (!ensure<R>(w, ip, 1)) return false;
            if (byte_at<R>(w, ip) != 0) break;
            t += 255;
            ++ip;
          }
          t += 15 + byte_at<R>(w, ip++);
        }
        t += 3;
      copy_literal_run:
        if (ip + t + 3 > ip_end || op + t > oend) return false;
        copy_literal(w, op, ip, t);
        op += t;
        ip += t;
        state = 4;
        continue;
      } else if (state != 4) {  // M1: 2-byte match after 1..3 trailing literals
        next = t & 3;
        if (!ensure<R>(w, ip, 1)) return false;
        m_pos = op - 1 - (t >> 2) - ((int64_t)byte_at<R>(w, ip++) << 2);
        if (m_pos < out0 || m_pos >= op || op + 2 > oend) return false;
        copy_match(w, op, op - m_pos, 2);
        op += 2;
        goto match_next;
      } else {  // M1 after a literal run: 3 bytes, offset 2049..3072
        next = t & 3;
        if (!ensure<R>(w, ip, 1)) return false;
        m_pos = op - (1 + 0x0800) - (t >> 2) - ((int64_t)byte_at<R>(w, ip++) << 2);
        t = 3;
      }
    } else if (t >= 64) {  // M2
      next = t & 3;
      if (!ensure<R>(w, ip, 1)) return false;
      m_pos = op - 1 - ((t >> 2) & 7) - ((int64_t)byte_at<R>(w, ip++) << 3);
      t = (t >> 5) - 1 + 2;
    } else if (t >= 32) {  // M3
      t = (t & 31) + 2;
      if (t == 2) {
        for (;;) {
          if (!ensure<R>(w, ip, 1)) return false;
          if (byte_at<R>(w, ip) != 0) break;
          t += 255;
          ++ip;
        }
        t += 31 + byte_at<R>(w, ip++);
      }
      if (!ensure<R>(w, ip, 2)) return false;
      next = (int64_t)byte_at<R>(w, ip) | ((int64_t)byte_at<R>(w, ip + 1) << 8);
      ip += 2;
      m_pos = op - 1 - (next >> 2);
      next &= 3;
    } else {  // M4 (16..31), or end of stream
      m_pos = op - ((t & 8) << 11);
      t = (t & 7) + 2;
      if (t == 2) {
        for (;;) {
          if (!ensure<R>(w, ip, 1)) return false;
          if (byte_at<R>(w, ip) != 0) break;
          t += 255;
          ++ip;
        }
        t += 7 + byte_at<R>(w, ip++);
      }
      if (!ensure<R>(w, ip, 2)) return false;
      next = (int64_t)byte_at<R>(w, ip) | ((int64_t)byte_at<R>(w, ip + 1) << 8);
      ip += 2;
      m_pos -= next >> 2;
      next &= 3;
      if (m_pos == op) {
        *produced = op - out0;
        return t == 3 && ip == ip_end;
      }
      m_pos -= 0x4000;
    }
    if (m_pos < out0 || m_pos >= op || op + t > oend) return false;
    copy_match(w, op, op - m_pos, t);
    op += t;
  match_next:
    state = next;
    t = next;
    if (ip + t + 3 > ip_end || op + t > oend) return false;
    copy_literal(w, op, ip, t);
    op += t;
    ip += t;
  }
}

__host__ __device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// ---- LZO1X, lean wave parse (launch_block_decode default for LZO). The r6 PMC pass of the kernels above
// on TeraSort data (profiles/r6/r6f_pmc_lzo_decode_register_vs_lds.md): ~20 scalar instructions per output
// byte with the LDS window and the same with the register window, i.e. the window reads were never the
// cost -- the per-byte 64-bit bounds/window checks, the per-token prefix test and the loop scaffolding of
// the 64-lane copies were. Here:
//   * positions are 32-bit offsets from the block's input / output base (a Hadoop block is < 2 GiB),
//   * a token's bytes come from one 4-byte peek of the register window (two v_readlane) instead of a
//     checked read per byte: every token of a valid LZO1X stream starts with >= 3 bytes left (the stream
//     ends with the 3-byte end marker and every literal check keeps that margin), so a token's fixed bytes
//     need no bounds check; only the zero-run length extensions check as they go,
//   * literals of up to 64 bytes are copied out of the register window with one ds_bpermute (no global
//     load, so no load-to-store wait on the parse's path), longer ones by the 64-lane vector copy,
//   * a match of up to 64 bytes is one masked byte move per lane,
//   * the prefix decode (clip) is a template parameter, so the full decode pays nothing for it.
struct LeanWin {
  uint32_t rw = 0;    // this lane's 4 bytes of the 256-byte window at base
  uint32_t base = 0;  // chunk-relative offset of window byte 0
  uint32_t lim = 0;   // bytes [ip, ip + n) are in the window while ip + n <= lim (0: empty)
};

__device__ __forceinline__ void lean_fill(LeanWin& w, const uint8_t* ib, uint32_t ip, uint32_t ip_end, int lane) {
  const uint32_t base = ip & ~3u;
  const uint32_t end = min(base + (uint32_t)kRegWin, ip_end);
  const uint32_t p = base + 4 * (uint32_t)lane;
  uint32_t v = 0;
  if (p + 4 <= end) {
    v = reinterpret_cast<const U32p*>(ib + p)->v;
  } else {
    for (uint32_t k = 0; k < 4; ++k)
      if (p + k < end) v |= (uint32_t)ib[p + k] << (8 * k);
  }
  w.rw = v;
  w.base = base;
  // the chunk's last window holds every remaining byte (zeros past the end): never refilled again
  w.lim = end == ip_end ? 0xFFFFFFFFu : end;
}

// Bytes ip .. ip+3, little-endian (bytes past the chunk end read as zero).
__device__ __forceinline__ uint32_t lean_peek4(LeanWin& w, const uint8_t* ib, uint32_t ip, uint32_t ip_end, int lane) {
  if (ip + 4 > w.lim) lean_fill(w, ib, ip, ip_end, lane);
  const uint32_t d = ip - w.base;
  const uint32_t i = (d >> 2) & 63;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)w.rw, (int)i);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)w.rw, (int)((i + 1) & 63));
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (d & 3)));
}

template <bool P>
__device__ __forceinline__ void lean_literal(LeanWin& w, const uint8_t* ib, uint8_t* ob, uint32_t op, uint32_t ip,
                                             uint32_t ip_end, uint32_t len, uint32_t clip, int lane) {
  if (P) {
    if (op >= clip) return;
    len = min(len, clip - op);
  }
  if (len == 0) return;
  if (len <= 64) {
    if (ip + len > w.lim) lean_fill(w, ib, ip, ip_end, lane);
    const uint32_t e = ip - w.base + (uint32_t)lane;  // window offset of this lane's byte
    const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(e & 0xFCu), (int)w.rw);
    if ((uint32_t)lane < len) ob[op + lane] = (uint8_t)(word >> (8 * (e & 3)));
  } else {
    wave_copy(ob + op, ib + ip, len, lane);
  }
}

template <bool P>
__device__ __forceinline__ void lean_match(uint8_t* ob, uint32_t op, uint32_t off, uint32_t len, uint32_t clip,
                                           uint32_t& flushed, int lane) {
  if (P) {
    if (op >= clip) return;
    len = min(len, clip - op);  // the source bytes below the clip were all written
  }
  const uint32_t src = op - off;
  if (src + min(off, len) > flushed) {  // reads bytes this wave stored since its last fence
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    flushed = op;
  }
  if (len <= 64) {
    if ((uint32_t)lane < len) ob[op + lane] = ob[src + (off >= len ? (uint32_t)lane : (uint32_t)lane % off)];
  } else if (off >= len) {
    wave_copy(ob + op, ob + src, len, lane);
  } else {
    for (uint32_t i = lane; i < len; i += 64) ob[op + i] = ob[src + i % off];
  }
}

// One LZO1X chunk [ip, ip_end) of the block at ib, output at ob + op (block-relative offsets).
template <bool P>
__device__ bool lzo_lean_chunk(const uint8_t* ib, uint8_t* ob, uint32_t ip, const uint32_t ip_end, uint32_t op,
                               const uint32_t oend, const uint32_t clip, uint32_t& flushed, const int lane,
                               uint32_t* produced) {
  LeanWin w;
  const uint32_t out0 = op;
  uint32_t t = 0, next = 0, state = 0, m_pos = 0, v = 0;
  if (ip + 3 > ip_end) return false;  // shortest stream: the end marker
  v = lean_peek4(w, ib, ip, ip_end, lane);
  if ((v & 0xFF) > 17) {
    t = (v & 0xFF) - 17;
    ++ip;
    if (t < 4) {
      next = t;
      goto match_next;
    }
    goto literal_run;
  }
  for (;;) {
    // here ip + 3 <= ip_end: the token byte and up to two more are in bounds
    if (P && op >= clip) {
      *produced = oend - out0;
      return true;
    }
    v = lean_peek4(w, ib, ip, ip_end, lane);
    t = v & 0xFF;
    if (t < 16) {
      if (state == 0) {
        ++ip;
        if (t == 0) {
          uint32_t b;
          for (;;) {
            if (ip >= ip_end) return false;
            b = lean_peek4(w, ib, ip, ip_end, lane) & 0xFF;
            if (b != 0) break;
            t += 255;
            ++ip;
          }
          t += 15 + b;
          ++ip;
        }
        t += 3;
      literal_run:
        if (ip + t + 3 > ip_end || op + t > oend) return false;
        lean_literal<P>(w, ib, ob, op, ip, ip_end, t, clip, lane);
        op += t;
        ip += t;
        state = 4;
        continue;
      } else if (state != 4) {  // M1: 2-byte match after 1..3 trailing literals
        next = t & 3;
        m_pos = op - 1 - (t >> 2) - (((v >> 8) & 0xFF) << 2);
        ip += 2;
        if (m_pos < out0 || m_pos >= op || op + 2 > oend) return false;
        lean_match<P>(ob, op, op - m_pos, 2, clip, flushed, lane);
        op += 2;
        goto match_next;
      } else {  // M1 after a literal run: 3 bytes, offset 2049..3072
        next = t & 3;
        m_pos = op - (1 + 0x0800) - (t >> 2) - (((v >> 8) & 0xFF) << 2);
        ip += 2;
        t = 3;
      }
    } else if (t >= 64) {  // M2
      next = t & 3;
      m_pos = op - 1 - ((t >> 2) & 7) - (((v >> 8) & 0xFF) << 3);
      ip += 2;
      t = (t >> 5) + 1;
    } else {  // M3 (32..63) / M4 (16..31, or the end of the stream)
      const bool m3 = t >= 32;
      const uint32_t lmask = m3 ? 31u : 7u;
      if (!m3) m_pos = op - ((t & 8) << 11);
      t = (t & lmask) + 2;
      if (t == 2) {  // zero-run length extension
        ++ip;
        uint32_t b;
        for (;;) {
          if (ip + 3 > ip_end) return false;  // this byte and the two offset bytes after the run
          b = lean_peek4(w, ib, ip, ip_end, lane) & 0xFF;
          if (b != 0) break;
          t += 255;
          ++ip;
        }
        t += lmask + b;
        ++ip;
        next = lean_peek4(w, ib, ip, ip_end, lane) & 0xFFFF;
        ip += 2;
      } else {
        next = (v >> 8) & 0xFFFF;
        ip += 3;
      }
      if (m3) {
        m_pos = op - 1 - (next >> 2);
        next &= 3;
      } else {
        m_pos -= next >> 2;
        next &= 3;
        if (m_pos == op) {
          *produced = op - out0;
          return t == 3 && ip == ip_end;
        }
        m_pos -= 0x4000;
      }
    }
    // m_pos below 0 wraps above op and fails the second test
    if (m_pos < out0 || m_pos >= op || op + t > oend) return false;
    lean_match<P>(ob, op, op - m_pos, t, clip, flushed, lane);
    op += t;
  match_next:
    state = next;
    t = next;
    if (ip + t + 3 > ip_end || op + t > oend) return false;
    lean_literal<P>(w, ib, ob, op, ip, ip_end, t, clip, lane);
    op += t;
    ip += t;
  }
}

template <bool P>
__global__ void __launch_bounds__(64 * kWavesPerBlock)
    lzo_lean_kernel(const uint8_t* in, uint8_t* out, const DecodeDesc* descs, int n, int* status, int64_t clip_in) {
  // wave-uniform by construction, but the compiler's divergence analysis cannot see through
  // threadIdx.x >> 6: say so, or every value derived from the descriptor -- the whole parse -- lives in
  // VGPRs with exec-masked branches instead of SGPRs and scalar branches
  const int b = blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (b >= n) return;
  const DecodeDesc d = descs[b];
  const int lane = threadIdx.x & 63;
  const uint8_t* ib = in + d.src;
  uint8_t* ob = out + d.dst;
  const int64_t ilen = d.src_end - d.src;
  bool ok = ilen >= 0 && ilen < (1ll << 31) && d.raw >= 0 && d.raw < (1ll << 31);
  const uint32_t ie = ok ? (uint32_t)ilen : 0, oend = ok ? (uint32_t)d.raw : 0;
  const uint32_t clip = P ? (uint32_t)min(clip_in, (int64_t)oend) : oend;
  uint32_t ip = 0, op = 0, flushed = 0;
  // one block = one or more [u32 BE compressed_len][chunk] records until its raw bytes are produced
  while (ok && op < oend) {
    if (P && op >= clip) return;  // prefix decode done
    if (ip + 4 > ie) {
      ok = false;
      break;
    }
    const uint32_t clen = be32(ib + ip);
    ip += 4;
    if (clen > ie - ip) {
      ok = false;
      break;
    }
    uint32_t produced = 0;
    ok = lzo_lean_chunk<P>(ib, ob, ip, ip + clen, op, oend, clip, flushed, lane, &produced);
    ip += clen;
    op += produced;
  }
  if (ok && (op != oend || ip != ie)) ok = false;
  if (!ok && lane == 0) atomicOr(status, 1);
}

// clip > 0: prefix decode. Only the first `clip` bytes of each block's output (at d.dst) are written and
// the decode stops once they are out; d.raw stays the block's full raw size for the format checks.
template <int kCodec, bool R>
__global__ void __launch_bounds__(64 * kWavesPerBlock)
    block_decode_kernel(const uint8_t* in, uint8_t* out, const DecodeDesc* descs, int n, int* status, int64_t clip) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[R ? 1 : kWavesPerBlock][R ? 16 : kWin + 16];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (see lzo_lean_kernel)
  const int b = blockIdx.x * kWavesPerBlock + wid;
  if (b >= n) return;
  const DecodeDesc d = descs[b];
  Wave w;
  w.in = in;
  w.out = out;
  w.win = lds[R ? 0 : wid];
  w.rw = 0;
  w.win_base = 0;
  w.win_end = 0;
  w.flushed = d.dst;
  w.lane = threadIdx.x & 63;
  int64_t ip = d.src, op = d.dst;
  const int64_t oend = d.dst + d.raw;
  w.prefix = clip > 0 && clip < d.raw;
  w.clip = w.prefix ? d.dst + clip : oend;
  bool ok = true;
  // one block = one or more [u32 BE compressed_len][chunk] records until its raw bytes are produced
  while (ok && op < oend) {
    if (w.prefix && op >= w.clip) return;  // prefix decode done
    if (ip + 4 > d.src_end) {
      ok = false;
      break;
    }
    const int64_t clen = (int64_t)be32(in + ip);
    ip += 4;
    if (ip + clen > d.src_end) {
      ok = false;
      break;
    }
    int64_t produced = 0;
    w.win_base = w.win_end = 0;
    ok = (kCodec == 1) ? snappy_chunk<R>(w, ip, ip + clen, op, oend, &produced)
                       : lzo_chunk<R>(w, ip, ip + clen, op, oend, &produced);
    ip += clen;
    op += produced;
  }
  if (ok && (op != oend || ip != d.src_end)) ok = false;
  if (!ok && w.lane == 0) atomicOr(status, 1);
}

// ---- LZO1X, one lane per block (launch_block_decode default for LZO; UDA_LZO_LANE=0: the wave-per-block
// kernel above). The wave-uniform parse spent ~20 scalar instructions per output byte on TeraSort data:
// random 10-byte keys and 26-letter values compress into 3-4 byte matches between 1-3 byte literal runs,
// so a 256 KiB block is ~60K tokens and every token paid the wave's whole scalar parse plus a 64-lane copy
// for a few bytes. Here each lane runs the state machine of its own block: 64 blocks advance one token
// per wave step, a token's bytes are copied by its lane (8-byte unaligned moves, a byte loop for the
// overlapping short-offset matches), and the input is read 8 bytes at a time into a per-lane register.
// A lane only ever reads back what it wrote itself, so no fence is needed between its copies.
struct __attribute__((packed, aligned(1))) U64p {
  uint64_t v;
};

struct LaneIn {  // the next input bytes of one lane, 8 at a time
  const uint8_t* in;
  int64_t end;     // one past the last readable byte of this block
  int64_t base = -8;
  uint64_t word = 0;
  __host__ __device__ __forceinline__ uint32_t at(int64_t ip) {
    const int64_t d = ip - base;
    if (d < 0 || d >= 8) {
      base = ip;
      if (ip + 8 <= end) {
        word = reinterpret_cast<const U64p*>(in + ip)->v;
      } else {
        word = 0;
        for (int k = 0; k < 8 && ip + k < end; ++k) word |= (uint64_t)in[ip + k] << (8 * k);
      }
      return (uint32_t)(word & 0xFF);
    }
    return (uint32_t)((word >> (8 * d)) & 0xFF);
  }
};

// dst[0, len) = src[0, len), non-overlapping or src >= dst + 8 behind (forward, 8 bytes per move)
__host__ __device__ __forceinline__ void lane_copy(uint8_t* dst, const uint8_t* src, int64_t len) {
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) reinterpret_cast<U64p*>(dst + i)->v = reinterpret_cast<const U64p*>(src + i)->v;
  for (; i < len; ++i) dst[i] = src[i];
}

__host__ __device__ __forceinline__ void lane_match(uint8_t* out, int64_t op, int64_t off, int64_t len) {
  if (off >= 8) {
    lane_copy(out + op, out + op - off, len);
  } else {
    for (int64_t i = 0; i < len; ++i) out[op + i] = out[op - off + i];
  }
}

// LZO1X chunk of one lane (csrc/codec/lzo.cc semantics, same bounds checks as lzo_chunk).
__host__ __device__ bool lzo_lane_chunk(const uint8_t* in, uint8_t* out, int64_t ip, int64_t ip_end, int64_t op, int64_t oend,
                               int64_t clip, bool prefix, int64_t* produced) {
  LaneIn r{in, ip_end};
  const int64_t out0 = op;
  int64_t t = 0, next = 0, state = 0, m_pos = 0;
  bool lit_first = false;
  if (ip >= ip_end) return false;
  auto lit = [&](int64_t len) {  // the bytes below the clip
    const int64_t n = len < clip - op ? len : clip - op;
    if (n > 0) lane_copy(out + op, in + ip, n);
  };
  auto match = [&](int64_t off, int64_t len) {
    const int64_t n = len < clip - op ? len : clip - op;
    if (n > 0) lane_match(out, op, off, n);
  };
  if (r.at(ip) > 17) {
    t = (int64_t)r.at(ip) - 17;
    ++ip;
    if (t < 4) {
      next = t;
      goto match_next;
    }
    lit_first = true;
  }
  for (;;) {
    if (prefix && op >= clip) {
      *produced = oend - out0;
      return true;
    }
    if (lit_first) {
      lit_first = false;
      goto copy_literal_run;
    }
    if (ip >= ip_end) return false;
    t = r.at(ip++);
    if (t < 16) {
      if (state == 0) {
        if (t == 0) {
          for (;;) {
            if (ip >= ip_end) return false;
            if (r.at(ip) != 0) break;
            t += 255;
            ++ip;
          }
          t += 15 + r.at(ip++);
        }
        t += 3;
      copy_literal_run:
        if (ip + t + 3 > ip_end || op + t > oend) return false;
        lit(t);
        op += t;
        ip += t;
        state = 4;
        continue;
      } else if (state != 4) {  // M1: 2-byte match after 1..3 trailing literals
        next = t & 3;
        if (ip >= ip_end) return false;
        m_pos = op - 1 - (t >> 2) - ((int64_t)r.at(ip++) << 2);
        if (m_pos < out0 || m_pos >= op || op + 2 > oend) return false;
        match(op - m_pos, 2);
        op += 2;
        goto match_next;
      } else {  // M1 after a literal run: 3 bytes, offset 2049..3072
        next = t & 3;
        if (ip >= ip_end) return false;
        m_pos = op - (1 + 0x0800) - (t >> 2) - ((int64_t)r.at(ip++) << 2);
        t = 3;
      }
    } else if (t >= 64) {  // M2
      next = t & 3;
      if (ip >= ip_end) return false;
      m_pos = op - 1 - ((t >> 2) & 7) - ((int64_t)r.at(ip++) << 3);
      t = (t >> 5) - 1 + 2;
    } else if (t >= 32) {  // M3
      t = (t & 31) + 2;
      if (t == 2) {
        for (;;) {
          if (ip >= ip_end) return false;
          if (r.at(ip) != 0) break;
          t += 255;
          ++ip;
        }
        t += 31 + r.at(ip++);
      }
      if (ip + 2 > ip_end) return false;
      next = (int64_t)r.at(ip) | ((int64_t)r.at(ip + 1) << 8);
      ip += 2;
      m_pos = op - 1 - (next >> 2);
      next &= 3;
    } else {  // M4 (16..31), or end of stream
      m_pos = op - ((t & 8) << 11);
      t = (t & 7) + 2;
      if (t == 2) {
        for (;;) {
          if (ip >= ip_end) return false;
          if (r.at(ip) != 0) break;
          t += 255;
          ++ip;
        }
        t += 7 + r.at(ip++);
      }
      if (ip + 2 > ip_end) return false;
      next = (int64_t)r.at(ip) | ((int64_t)r.at(ip + 1) << 8);
      ip += 2;
      m_pos -= next >> 2;
      next &= 3;
      if (m_pos == op) {
        *produced = op - out0;
        return t == 3 && ip == ip_end;
      }
      m_pos -= 0x4000;
    }
    if (m_pos < out0 || m_pos >= op || op + t > oend) return false;
    match(op - m_pos, t);
    op += t;
  match_next:
    state = next;
    t = next;
    if (ip + t + 3 > ip_end || op + t > oend) return false;
    lit(t);
    op += t;
    ip += t;
  }
}

__global__ void __launch_bounds__(64) lzo_lane_kernel(const uint8_t* in, uint8_t* out, const DecodeDesc* descs, int n,
                                                       int* status, int64_t clip_in) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const DecodeDesc d = descs[b];
  int64_t ip = d.src, op = d.dst;
  const int64_t oend = d.dst + d.raw;
  const bool prefix = clip_in > 0 && clip_in < d.raw;
  const int64_t clip = prefix ? d.dst + clip_in : oend;
  bool ok = true;
  while (ok && op < oend) {
    if (prefix && op >= clip) return;
    if (ip + 4 > d.src_end) {
      ok = false;
      break;
    }
    const int64_t clen = (int64_t)be32(in + ip);
    ip += 4;
    if (ip + clen > d.src_end) {
      ok = false;
      break;
    }
    int64_t produced = 0;
    ok = lzo_lane_chunk(in, out, ip, ip + clen, op, oend, clip, prefix, &produced);
    ip += clen;
    op += produced;
  }
  if (ok && (op != oend || ip != d.src_end)) ok = false;
  if (!ok) atomicOr(status, 1);
}

}  // namespace

// The lane kernel's per-block decode run on the host over one block-compressed stream (tests: the same
// code path the device lanes run, checked on a machine without a GPU). false on a corrupt block.
bool lzo_lane_decode_host(const uint8_t* in, int64_t n, uint8_t* out, int64_t out_cap, int64_t* out_len) {
  int64_t i = 0, op = 0;
  while (i < n) {
    if (i + 4 > n) return false;
    const int64_t block_raw = (int64_t)be32(in + i);
    i += 4;
    if (block_raw == 0) continue;
    if (op + block_raw > out_cap) return false;
    const int64_t oend = op + block_raw;
    while (op < oend) {
      if (i + 4 > n) return false;
      const int64_t clen = (int64_t)be32(in + i);
      i += 4;
      if (i + clen > n) return false;
      int64_t produced = 0;
      if (!lzo_lane_chunk(in, out, i, i + clen, op, oend, oend, false, &produced)) return false;
      i += clen;
      op += produced;
    }
    if (op != oend) return false;
  }
  *out_len = op;
  return true;
}

// Framing walk of device-resident block-compressed streams (one lane per stream, following the
// 4-byte headers; a header read per chunk). Pass 1 (out == nullptr): blocks and raw bytes per
// stream. Pass 2: the decode descriptors, src/src_end as absolute device addresses (decode with a
// null input base), dst at raw_first[s] + the stream's earlier raw bytes. status[s] = 1 when the
// framing is not resolvable without decoding (the host planner's `false`).
__global__ void __launch_bounds__(64) frame_streams_kernel(const uint8_t* const* ptrs, const int64_t* lens, int nstreams,
                                                           int codec, const int64_t* desc_first, const int64_t* raw_first,
                                                           int64_t* nblocks, int64_t* raw, DecodeDesc* out, int* status) {
  const int sidx = blockIdx.x * blockDim.x + threadIdx.x;
  if (sidx >= nstreams) return;
  const uint8_t* p = ptrs[sidx];
  const int64_t n = lens[sidx];
  int64_t i = 0, blocks = 0, rsum = 0;
  int bad = 0;
  while (i < n && !bad) {
    if (i + 4 > n) {
      bad = 1;
      break;
    }
    const int64_t block_raw = (int64_t)be32(p + i);
    i += 4;
    if (block_raw == 0) continue;
    const int64_t start = i;
    int64_t left = block_raw;
    while (left > 0) {
      if (i + 4 > n) {
        bad = 1;
        break;
      }
      const int64_t clen = (int64_t)be32(p + i);
      if (i + 4 + clen > n) {
        bad = 1;
        break;
      }
      int64_t produced = left;  // LZO: one chunk produces the whole block
      if (codec == 1) {         // Snappy: the chunk's uncompressed-length varint
        uint64_t u = 0;
        int sh = 0, k = 0;
        for (; k < 5 && k < clen; ++k) {
          const uint8_t b = p[i + 4 + k];
          u |= (uint64_t)(b & 0x7F) << sh;
          sh += 7;
          if (!(b & 0x80)) break;
        }
        if (k >= 5 || k >= clen) {
          bad = 1;
          break;
        }
        produced = (int64_t)u;
        if (produced > left || produced == 0) {
          bad = 1;
          break;
        }
      }
      i += 4 + clen;
      left -= produced;
    }
    if (bad) break;
    if (out) {
      DecodeDesc d;
      d.src = (int64_t)(uintptr_t)(p + start);
      d.src_end = (int64_t)(uintptr_t)(p + i);
      d.dst = raw_first[sidx] + rsum;
      d.raw = block_raw;
      out[desc_first[sidx] + blocks] = d;
    }
    ++blocks;
    rsum += block_raw;
  }
  if (!out) {
    nblocks[sidx] = blocks;
    raw[sidx] = rsum;
  }
  if (bad) status[sidx] = 1;
}

void launch_frame_streams(const uint8_t* const* ptrs, const int64_t* lens, int nstreams, int codec,
                          const int64_t* desc_first, const int64_t* raw_first, int64_t* nblocks, int64_t* raw,
                          DecodeDesc* out, int* status, hipStream_t s) {
  if (nstreams <= 0) return;
  hipLaunchKernelGGL(frame_streams_kernel, dim3((unsigned)((nstreams + 63) / 64)), dim3(64), 0, s, ptrs, lens, nstreams,
                     codec, desc_first, raw_first, nblocks, raw, out, status);
}

void launch_block_decode(int codec, const uint8_t* in, uint8_t* out, const DecodeDesc* descs, int n, int* status,
                         hipStream_t s, int64_t clip) {
  if (n <= 0) return;
  const int grid = (n + kWavesPerBlock - 1) / kWavesPerBlock;
  // read per launch: tests compare the kernels in one process
  const char* le = std::getenv("UDA_LZO_LANE");  // 1: one lane per LZO block (too few blocks per round to hide latency)
  const bool lzo_lane = le && std::atoi(le) != 0;
  // "lds": the LDS window of round 5; "reg": the register window with the per-byte parse (LZO; Snappy's
  // default); unset: the lean LZO parse
  const char* we = std::getenv("UDA_DECODE_WINDOW");
  const bool reg = !we || std::string(we) != "lds";
  const bool lean = !we || !*we;
  if (codec == 2 && lean && !lzo_lane) {
    if (clip > 0)
      lzo_lean_kernel<true><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
    else
      lzo_lean_kernel<false><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
  } else if (codec == 1 && reg)
    block_decode_kernel<1, true><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
  else if (codec == 1)
    block_decode_kernel<1, false><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
  else if (lzo_lane)
    // one wave per workgroup: a round's few hundred waves spread over the CUs (each with its own L1 for
    // its 64 lanes' input and output streams) instead of packing four on one CU
    lzo_lane_kernel<<<(n + 63) / 64, 64, 0, s>>>(in, out, descs, n, status, clip);
  else if (reg)
    block_decode_kernel<2, true><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
  else
    block_decode_kernel<2, false><<<grid, 64 * kWavesPerBlock, 0, s>>>(in, out, descs, n, status, clip);
}

}  // namespace gpu
}  // namespace uda
