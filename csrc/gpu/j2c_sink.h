// Native stand-in for the Java reducer that consumes the merged stream: per reduce task, every
// delivered buffer is copied into a 1 MiB KVBuf (two of them, alternating) and its records are
// walked by their VInt key/value lengths, exactly the work UdaPluginRT.dataFromUda and
// J2CQueue.next do (plugins/shared/com/mellanox/hadoop/mapred/UdaPlugin.java:369-402,498-538).
// Each reduce task is consumed by its own thread (the engine's per-reducer consumer), so the sink
// keeps per-reducer state only and needs no locks on the hot path.
//
// It also validates the delivery contract: every buffer holds whole records, is at most
// kv_buf_bytes long, and each reducer's stream ends with exactly one EOF marker (-1, -1).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "uda/vint.h"

namespace uda {
namespace gpu {

class J2CSink {
 public:
  enum Error : int { kOk = 0, kTooLong = 1, kBadFraming = 2, kAfterEof = 3 };

  J2CSink(int reducers, int64_t kv_buf_bytes) : kv_(kv_buf_bytes), st_(reducers) {
    for (auto& s : st_) {
      s.buf[0].reset(new uint8_t[(size_t)kv_buf_bytes]);
      s.buf[1].reset(new uint8_t[(size_t)kv_buf_bytes]);
    }
  }

  int reducers() const { return (int)st_.size(); }

  // Called from reducer r's consumer thread only.
  int consume(int r, const uint8_t* data, int64_t len) {
    State& s = st_[(size_t)r];
    if (len > kv_) return fail(s, kTooLong);
    if (s.eof) return fail(s, kAfterEof);
    uint8_t* kb = s.buf[s.cur].get();
    s.cur ^= 1;
    std::memcpy(kb, data, (size_t)len);  // dataFromUda: DirectByteBuffer -> KVBuf
    int64_t p = 0, recs = 0;
    const bool order = check_order_;
    if (!order) {  // fast path of the walk below: both VInt headers one byte (lengths < 128)
      while (p + 2 <= len) {
        const int8_t k1 = (int8_t)kb[p], v1 = (int8_t)kb[p + 1];
        if ((k1 | v1) < 0) break;  // multi-byte header or the EOF marker: general decoder
        const int64_t next = p + 2 + k1 + v1;
        if (next > len) return fail(s, kBadFraming);
        s.key_bytes += k1;
        ++recs;
        p = next;
      }
    }
    while (p < len) {  // J2CQueue.next: readVInt key length, readVInt value length, skip bytes
      int64_t kl = 0, vl = 0;
      const int a = vint_decode(kb + p, (size_t)(len - p), &kl);
      if (a <= 0) return fail(s, kBadFraming);
      const int b = vint_decode(kb + p + a, (size_t)(len - p - a), &vl);
      if (b <= 0) return fail(s, kBadFraming);
      if (kl == -1 && vl == -1) {
        if (p + a + b != len) return fail(s, kBadFraming);
        s.eof = true;
        p = len;
        break;
      }
      if (kl < 0 || vl < 0) return fail(s, kBadFraming);
      if (p + a + b + kl + vl > len) return fail(s, kBadFraming);
      if (order) {  // keys ascend within a reducer (content bytes after the key class's length prefix)
        const uint8_t* k = kb + p + a + b;
        int64_t ko = 0;
        if (key_kind_ == 1 && kl > 0) ko = std::min<int64_t>(kl, vint_decode_size((int)(int8_t)k[0]));  // Text
        if (key_kind_ == 2) ko = std::min<int64_t>(kl, 4);                                              // BytesWritable
        k += ko;
        const int kn = (int)std::min<int64_t>(kl - ko, (int64_t)sizeof(s.last_key));
        if (s.has_last) {
          const int n = std::min(kn, s.last_len);
          const int c = std::memcmp(s.last_key, k, (size_t)n);
          if (c > 0 || (c == 0 && s.last_len > kn)) ++s.order_errors;
        }
        std::memcpy(s.last_key, k, (size_t)kn);
        s.last_len = kn;
        s.has_last = true;
      }
      p += a + b + kl + vl;
      s.key_bytes += kl;
      ++recs;
    }
    if (p != len) return fail(s, kBadFraming);
    s.records += recs;
    s.bytes += len;
    s.buffers += 1;
    return kOk;
  }

  void reset() {
    for (auto& s : st_) {
      s.records = s.bytes = s.buffers = s.key_bytes = s.order_errors = 0;
      s.eof = false;
      s.has_last = false;
      s.error = kOk;
    }
  }
  // Also check that keys ascend within every reducer (the first 256 bytes, see set_key_kind). Raw
  // serialized bytes are the key order for fixed-length keys such as TeraSort's 10-byte Text keys.
  void set_check_order(bool on) { check_order_ = on; }
  // Key class of the order check: 0 raw serialized bytes (default), 1 Text, 2 BytesWritable: the
  // comparator's content bytes (first 256), then their length.
  void set_key_kind(int k) { key_kind_ = k; }
  int64_t order_errors(int r) const { return st_[(size_t)r].order_errors; }
  int64_t records(int r) const { return st_[(size_t)r].records; }
  int64_t bytes(int r) const { return st_[(size_t)r].bytes; }
  int64_t buffers(int r) const { return st_[(size_t)r].buffers; }
  bool eof(int r) const { return st_[(size_t)r].eof; }
  int error(int r) const { return st_[(size_t)r].error; }

 private:
  struct alignas(64) State {
    std::unique_ptr<uint8_t[]> buf[2];
    int cur = 0;
    int64_t records = 0, bytes = 0, buffers = 0, key_bytes = 0, order_errors = 0;
    bool eof = false;
    int error = kOk;
    bool has_last = false;
    int last_len = 0;
    uint8_t last_key[256];
  };
  static int fail(State& s, int e) {
    if (s.error == kOk) s.error = e;
    return e;
  }
  int64_t kv_;
  bool check_order_ = false;
  int key_kind_ = 0;
  std::vector<State> st_;
};

}  // namespace gpu
}  // namespace uda
