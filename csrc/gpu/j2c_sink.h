// Native stand-in for the Java reducer that consumes the merged stream: per reduce task, every
// delivered buffer is copied into a 1 MiB KVBuf (two of them, alternating) and its records are
// walked by their VInt key/value lengths, exactly the work UdaPluginRT.dataFromUda and
// J2CQueue.next do (plugins/shared/com/mellanox/hadoop/mapred/UdaPlugin.java:369-402,456-538).
//
// Threads, as in the plugin: dataFromUda runs on the thread that delivers the buffer (UDA's merge
// thread calling into the JVM) and only copies it into the next free KVBuf; the reduce task's own
// thread (J2CQueue.next) walks the KVBufs in order and hands each back once walked (the
// kv_buf_recv_ready / kv_buf_redc_ready handshake, kv_buf_num = 2). So a task's copy and walk overlap.
// `threaded = false` runs the walk inline in consume() (one thread per task does both).
//
// It also validates the delivery contract: every buffer holds whole records, is at most
// kv_buf_bytes long, and each reducer's stream ends with exactly one EOF marker (-1, -1).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "uda/vint.h"

namespace uda {
namespace gpu {

class J2CSink {
 public:
  enum Error : int { kOk = 0, kTooLong = 1, kBadFraming = 2, kAfterEof = 3 };

  // Default inline; UDA_J2C_THREADS=1 walks on the reduce task's own thread. Measured on MI355X boxes
  // (profiles/r3_j2c_threads_ab.md): the copy out of the SDMA-written ring, not the walk, bounds a
  // task (~25 GB/s per thread), so the split gains 9 % on the skewed config #5 task and loses on a
  // single out-of-cache stream (the walker reads the KVBuf from the copying core's cache).
  static bool default_threaded() {
    const char* e = std::getenv("UDA_J2C_THREADS");
    return e && std::atoi(e) != 0;
  }
  J2CSink(int reducers, int64_t kv_buf_bytes, bool threaded = default_threaded())
      : kv_(kv_buf_bytes), threaded_(threaded) {
    st_.reserve((size_t)reducers);
    for (int r = 0; r < reducers; ++r) {
      st_.emplace_back(new State);
      State& s = *st_.back();
      s.buf[0].reset(new uint8_t[(size_t)kv_buf_bytes]);
      s.buf[1].reset(new uint8_t[(size_t)kv_buf_bytes]);
    }
    if (threaded_)
      for (int r = 0; r < reducers; ++r) st_[(size_t)r]->walker = std::thread([this, r] { walk_loop(r); });
  }
  ~J2CSink() {
    for (auto& sp : st_) {
      std::lock_guard<std::mutex> g(sp->mu);
      sp->stop = true;
      sp->cv.notify_all();
    }
    for (auto& sp : st_)
      if (sp->walker.joinable()) sp->walker.join();
  }
  J2CSink(const J2CSink&) = delete;
  J2CSink& operator=(const J2CSink&) = delete;

  int reducers() const { return (int)st_.size(); }
  bool threaded() const { return threaded_; }

  // dataFromUda for reducer r (one delivering thread per reducer at a time). Threaded: returns once the
  // buffer is copied into a KVBuf; a walk error of an earlier buffer is returned by a later call.
  int consume(int r, const uint8_t* data, int64_t len) {
    State& s = *st_[(size_t)r];
    if (len > kv_) return fail(s, kTooLong);
    if (!threaded_) {
      if (s.eof) return fail(s, kAfterEof);
      uint8_t* kb = s.buf[s.cur].get();
      s.cur ^= 1;
      std::memcpy(kb, data, (size_t)len);  // dataFromUda: DirectByteBuffer -> KVBuf
      return walk(r, s, kb, len);
    }
    const int i = s.cur;
    {
      std::unique_lock<std::mutex> lk(s.mu);
      s.cv.wait(lk, [&] { return !s.full[i]; });  // kv_buf_recv_ready
    }
    std::memcpy(s.buf[i].get(), data, (size_t)len);
    {
      std::lock_guard<std::mutex> g(s.mu);
      s.len[i] = len;
      s.full[i] = true;  // kv_buf_redc_ready
      ++s.handed;
    }
    s.cv.notify_all();
    s.cur ^= 1;
    return s.error.load(std::memory_order_relaxed);
  }

  // Every buffer handed over so far has been walked (threaded mode; no-op inline).
  void flush() {
    if (!threaded_) return;
    for (auto& sp : st_) {
      std::unique_lock<std::mutex> lk(sp->mu);
      sp->cv.wait(lk, [&] { return sp->walked == sp->handed; });
    }
  }
  // Called by the walking thread once reducer r's EOF marker was walked.
  void set_on_eof(std::function<void(int)> fn) { on_eof_ = std::move(fn); }

  void reset() {
    flush();
    for (auto& sp : st_) {
      State& s = *sp;
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
  // Readers of the walk results: call flush() first in threaded mode.
  int64_t order_errors(int r) const { return st_[(size_t)r]->order_errors; }
  int64_t records(int r) const { return st_[(size_t)r]->records; }
  int64_t bytes(int r) const { return st_[(size_t)r]->bytes; }
  int64_t buffers(int r) const { return st_[(size_t)r]->buffers; }
  bool eof(int r) const { return st_[(size_t)r]->eof; }
  int error(int r) const { return st_[(size_t)r]->error.load(); }

 private:
  struct alignas(64) State {
    std::unique_ptr<uint8_t[]> buf[2];
    int cur = 0;  // next KVBuf dataFromUda fills
    // handshake (threaded mode)
    std::mutex mu;
    std::condition_variable cv;
    bool full[2] = {false, false};
    int64_t len[2] = {0, 0};
    int64_t handed = 0, walked = 0;
    bool stop = false;
    std::thread walker;
    // walk results (written by the walking thread)
    int64_t records = 0, bytes = 0, buffers = 0, key_bytes = 0, order_errors = 0;
    std::atomic<bool> eof{false};
    std::atomic<int> error{kOk};
    bool has_last = false;
    int last_len = 0;
    uint8_t last_key[256];
  };
  static int fail(State& s, int e) {
    int expect = kOk;
    s.error.compare_exchange_strong(expect, e);
    return e;
  }

  // J2CQueue.next over one KVBuf: readVInt key length, readVInt value length, skip the bytes.
  int walk(int r, State& s, const uint8_t* kb, int64_t len) {
    if (s.eof) return fail(s, kAfterEof);
    int64_t p = 0, recs = 0;
    const bool order = check_order_;
    if (!order) {  // fast path of the walk below: both VInt headers one byte (lengths < 128)
      int64_t keyb = 0;  // locals: a store through `s` may alias the byte buffer and pin every load
      while (p + 2 <= len) {
        const int8_t k1 = (int8_t)kb[p], v1 = (int8_t)kb[p + 1];
        if ((k1 | v1) < 0) break;  // multi-byte header or the EOF marker: general decoder
        const int64_t next = p + 2 + k1 + v1;
        if (next > len) return fail(s, kBadFraming);
        keyb += k1;
        ++recs;
        p = next;
      }
      s.key_bytes += keyb;
    }
    while (p < len) {
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
    if (s.eof && on_eof_) on_eof_(r);
    return s.error.load(std::memory_order_relaxed);
  }

  // The reduce task's thread: walk the KVBufs in fill order, hand each back when done.
  void walk_loop(int r) {
    State& s = *st_[(size_t)r];
    int i = 0;
    for (;;) {
      int64_t len;
      {
        std::unique_lock<std::mutex> lk(s.mu);
        s.cv.wait(lk, [&] { return s.full[i] || s.stop; });
        if (!s.full[i]) return;  // stopped with nothing left
        len = s.len[i];
      }
      walk(r, s, s.buf[i].get(), len);
      {
        std::lock_guard<std::mutex> g(s.mu);
        s.full[i] = false;
        ++s.walked;
      }
      s.cv.notify_all();
      i ^= 1;
    }
  }

  int64_t kv_;
  bool threaded_;
  bool check_order_ = false;
  int key_kind_ = 0;
  std::function<void(int)> on_eof_;
  std::vector<std::unique_ptr<State>> st_;
};

}  // namespace gpu
}  // namespace uda
