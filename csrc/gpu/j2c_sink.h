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
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
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
  // The reduce task's stand-in (C ABI bench, uda_reduce_task): the plugin's own shape, two threads
  // pinned to one last-level cache, unless UDA_J2C_THREADS=0. Config #5 at 100 GB, whose skewed task is
  // consumer-bound: 40.1 GB/s against 29.6 inline (profiles/r5/r5k_sec100_j2c.log).
  static bool plugin_threaded() {
    const char* e = std::getenv("UDA_J2C_THREADS");
    return !e || std::atoi(e) != 0;
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
    // UDA_J2C_PIN: l3 (default) = the walker and the copying thread share the copier's last-level cache
    // (the walker reads the KVBuf the copier just wrote); none = leave both to the scheduler
    const char* pin = std::getenv("UDA_J2C_PIN");
    pin_l3_ = !(pin && std::string(pin) == "none");
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
    if (s.handed == 0) place(s);
    if ((s.handed & 63) == 0) sample_cpu(s.copier_cpus);
    // kv_buf_recv_ready: the walker usually hands a KVBuf back within microseconds, sooner than a
    // sleeping thread is woken, so spin a little before blocking
    if (!spin_until([&] { return !s.full[i].load(std::memory_order_acquire); })) {
      std::unique_lock<std::mutex> lk(s.mu);
      ++s.copier_blocks;
      s.cv.wait(lk, [&] { return !s.full[i].load(); });
    }
    std::memcpy(s.buf[i].get(), data, (size_t)len);
    {
      std::lock_guard<std::mutex> g(s.mu);
      s.len[i] = len;
      s.full[i].store(true, std::memory_order_release);  // kv_buf_redc_ready
      ++s.handed;
    }
    if (s.walker_waiting.load()) s.cv.notify_all();
    s.cur ^= 1;
    return s.error.load(std::memory_order_relaxed);
  }

  // Where reducer r's copier and walker ran (threaded mode): CPUs, last-level caches and NUMA nodes
  // seen in samples, and how often each side had to block (the handshake's sleeps).
  std::string placement_json(int r) const {
    const State& s = *st_[(size_t)r];
    std::lock_guard<std::mutex> g(s.mu);
    auto desc = [](const std::map<int, int64_t>& cpus) {
      std::set<int> l3, node;
      for (auto& kv : cpus) {
        l3.insert(cpu_l3(kv.first));
        node.insert(cpu_node(kv.first));
      }
      std::string o = "{\"cpus\":" + std::to_string(cpus.size()) + ",\"l3\":[";
      bool first = true;
      for (int x : l3) {
        o += (first ? "" : ",") + std::to_string(x);
        first = false;
      }
      o += "],\"nodes\":[";
      first = true;
      for (int x : node) {
        o += (first ? "" : ",") + std::to_string(x);
        first = false;
      }
      return o + "]}";
    };
    return "{\"threaded\":" + std::string(threaded_ ? "true" : "false") + ",\"pinned_l3\":" +
           std::to_string(s.pinned_l3) + ",\"copier\":" + desc(s.copier_cpus) + ",\"walker\":" +
           desc(s.walker_cpus) + ",\"copier_blocks\":" + std::to_string(s.copier_blocks) +
           ",\"walker_blocks\":" + std::to_string(s.walker_blocks) + "}";
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
    mutable std::mutex mu;
    std::condition_variable cv;
    std::atomic<bool> full[2] = {{false}, {false}};
    int64_t len[2] = {0, 0};
    int64_t handed = 0, walked = 0;
    bool stop = false;
    std::atomic<bool> walker_waiting{false};
    std::thread walker;
    // placement (sampled every 64 buffers) and handshake sleeps
    std::map<int, int64_t> copier_cpus, walker_cpus;
    int64_t copier_blocks = 0, walker_blocks = 0;
    int pinned_l3 = -1;
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
    int64_t n = 0;
    for (;;) {
      int64_t len;
      if (!spin_until([&] { return s.full[i].load(std::memory_order_acquire); })) {
        std::unique_lock<std::mutex> lk(s.mu);
        if (!s.full[i].load()) ++s.walker_blocks;
        s.walker_waiting.store(true);
        s.cv.wait(lk, [&] { return s.full[i].load() || s.stop; });
        s.walker_waiting.store(false);
        if (!s.full[i].load()) return;  // stopped with nothing left
      }
      {
        std::lock_guard<std::mutex> g(s.mu);
        len = s.len[i];
        if ((n++ & 63) == 0) sample_cpu(s.walker_cpus);
      }
      walk(r, s, s.buf[i].get(), len);
      {
        std::lock_guard<std::mutex> g(s.mu);
        s.full[i].store(false, std::memory_order_release);
        ++s.walked;
      }
      s.cv.notify_all();  // a copier may block on this KVBuf, or flush() wait for the walk
      i ^= 1;
    }
  }

  // Spin up to ~50 us for pred(); false: the caller blocks.
  template <typename P>
  static bool spin_until(P pred) {
    if (pred()) return true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; ++k) {
      if (pred()) return true;
      if ((k & 31) == 31 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50)) return false;
      __builtin_ia32_pause();
    }
  }

  static void sample_cpu(std::map<int, int64_t>& m) {  // caller holds the state's lock or owns the map
    const int c = sched_getcpu();
    if (c >= 0) m[c]++;
  }
  static int read_int(const std::string& path) {
    std::ifstream f(path);
    int v = -1;
    if (f) f >> v;
    return v;
  }
  static int cpu_l3(int cpu) { return read_int("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache/index3/id"); }
  static int cpu_node(int cpu) {
    for (int n = 0; n < 64; ++n) {
      std::ifstream g("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
      if (!g) continue;
      // the node's CPU list "a-b,c-d"
      std::string list;
      std::getline(g, list);
      for (size_t b = 0; b < list.size();) {
        size_t e = list.find(',', b);
        if (e == std::string::npos) e = list.size();
        const std::string r = list.substr(b, e - b);
        const size_t dash = r.find('-');
        const int lo = std::atoi(r.c_str()), hi = dash == std::string::npos ? lo : std::atoi(r.c_str() + dash + 1);
        if (cpu >= lo && cpu <= hi) return n;
        b = e + 1;
      }
    }
    return -1;
  }
  // The CPUs sharing `cpu`'s last-level cache (empty if the host does not say).
  static std::vector<int> l3_cpus(int cpu) {
    std::ifstream f("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/cache/index3/shared_cpu_list");
    std::vector<int> v;
    std::string list;
    if (!f || !std::getline(f, list)) return v;
    for (size_t b = 0; b < list.size();) {
      size_t e = list.find(',', b);
      if (e == std::string::npos) e = list.size();
      const std::string r = list.substr(b, e - b);
      const size_t dash = r.find('-');
      const int lo = std::atoi(r.c_str()), hi = dash == std::string::npos ? lo : std::atoi(r.c_str() + dash + 1);
      for (int c = lo; c <= hi; ++c) v.push_back(c);
      b = e + 1;
    }
    return v;
  }
  // First buffer of reducer r: the copying thread and the walker move onto the copier's last-level
  // cache domain (both stay free to move within it), so the KVBuf the copier wrote is read from that
  // cache instead of across the fabric or from DRAM.
  void place(State& s) {
    if (!threaded_ || !pin_l3_) return;
    const int c = sched_getcpu();
    if (c < 0) return;
    // within the thread's own placement (a GPU's consumer slice of its NUMA node, uda/topology.h): the
    // L3 domain is narrowed to it, never widened past it into another GPU's slice
    cpu_set_t mine;
    if (pthread_getaffinity_np(pthread_self(), sizeof(mine), &mine) != 0) return;
    std::vector<int> cpus;
    for (int x : l3_cpus(c))
      if (x >= 0 && x < CPU_SETSIZE && CPU_ISSET(x, &mine)) cpus.push_back(x);
    if (cpus.size() < 2) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int x : cpus) CPU_SET(x, &set);
    if (pthread_setaffinity_np(pthread_self(), sizeof(set), &set) != 0) return;
    if (s.walker.joinable()) (void)pthread_setaffinity_np(s.walker.native_handle(), sizeof(set), &set);
    s.pinned_l3 = cpu_l3(c);
  }

  int64_t kv_;
  bool threaded_;
  bool pin_l3_ = true;
  bool check_order_ = false;
  int key_kind_ = 0;
  std::function<void(int)> on_eof_;
  std::vector<std::unique_ptr<State>> st_;
};

}  // namespace gpu
}  // namespace uda
