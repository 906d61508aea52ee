// NetMerger GPU backend (mapred.uda.merge.backend=gpu).
//
// Online (the reduce input fits the device budget): every fetched MOF partition is staged in HBM
// (compressed partitions cross PCIe compressed and are decoded there by the F6 kernels), the whole
// input is merged by the generic HIP merge tree (csrc/gpu/generic.hip) and streamed back to the
// host reducer through dataFromUda in whole-record buffers.
//
// Hybrid (input larger than the budget, mapred.uda.gpu.merge.bytes): the reference's two-level
// merge (merge_hybrid, src/Merger/MergeManager.cc:195-290) re-planned for a device:
//   LPQ  (disk tier, or mapred.uda.gpu.hybrid.direct=0) MOFs are grouped as they arrive; each group
//        is merged on the GPU and spilled to the local dirs through AsyncIO (io_uring) or to DRAM,
//        with a sparse index: the key at every record boundary the merge placed <= 256 KiB apart.
//        DRAM tier by default: no LPQ level; the fetched partitions are the runs, indexed the same
//        way by the drain threads (direct RPQ, see merge_gpu).
//   RPQ  instead of a streaming heap over the runs, the key space is cut into rounds from the
//        sparse indices (splitters every ~budget/2 bytes); for each round the matching byte range
//        of every run is copied to HBM and merged on the GPU in one go. Records equal to a splitter
//        all fall in the later round, in every run, so ties keep run order.
// Reference counterpart of the online path: merge_online (MergeManager.cc:184-193).
#include <fcntl.h>
#include <sys/stat.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <ctime>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <future>
#include <random>
#include <set>
#include <thread>

#include "../gpu/block_decoder.h"
#include "../gpu/device_ptr.h"
#include "../gpu/device_reduce.h"
#include "../gpu/device_engine.h"
#include "../gpu/generic_merger.h"
#include "../gpu/generic_rounds.h"
#include "../gpu/hbm_ledger.h"
#include "../gpu/sdma.h"
#include "reduce_task.h"
#include "uda/aio.h"
#include "uda/fault.h"
#include "uda/compare.h"
#include "uda/ifile.h"
#include "uda/log.h"
#include "uda/safe_file.h"
#include "uda/topology.h"
#include "uda/trace.h"

namespace uda {

namespace {

constexpr int64_t kSampleSpacing = 256 << 10;  // LPQ sparse-index granularity

struct DeviceMergeOut {
  int64_t bytes = 0;           // merged records (no EOF), resident in the workspace's `out`
  std::vector<int64_t> cuts;   // whole-record boundaries, <= the requested spacing apart
  int64_t records = 0;
  int64_t decoded_blocks = 0;
};

constexpr int64_t kPieceBytes = 64 << 20;  // D2H piece of the pinned double buffer (hipMemcpy fallback)
// stream_out's SDMA ring: a skewed task's delivery is the job's long pole (config #5: 60 GB in one task),
// and two 64 MiB pieces through hipMemcpyAsync left its consumer waiting on D2H for 815 of 2742 ms while
// 15 other tasks shared the link. Eight pieces of 16 MiB queued on the SDMA engines keep up to 128 MiB of
// the task's output moving ahead of its consumer, as the TeraSort delivery does (device_reduce.cc).
// (UDA_OUT_SLOTS / UDA_OUT_PIECE_MB: A/B of the ring's geometry)
const int kOutSlots = [] {
  const char* e = std::getenv("UDA_OUT_SLOTS");
  return e ? std::max(2, std::min(64, std::atoi(e))) : 8;
}();
const int64_t kOutPiece = [] {
  const char* e = std::getenv("UDA_OUT_PIECE_MB");
  return (e ? std::max<int64_t>(1, std::min<int64_t>(256, std::atoll(e))) : 16) << 20;
}();

// One merged LPQ output, resident in host memory or in a spill file.
struct SpillRun {
  uint8_t* mem = nullptr;         // host tier: pinned (spill arena)
  std::string path;
  int fd = -1;
  int64_t bytes = 0;
  std::vector<int64_t> cut;       // record-boundary offsets (first 0)
  std::vector<std::string> key;   // key bytes of the record at each cut
};

// Device buffers reused across the merges of one reduce task (LPQ groups, RPQ rounds): HBM is
// allocated once at the high-water mark instead of per merge (hipMalloc/hipFree of GBs costs ms and
// hipFree synchronizes the device).
struct DeviceWorkspace {
  int64_t pool_key = 0;  // input bytes of the task that last used it (DevicePool::acquire_fit)
  gpu::DeviceBuffer in, out, packed, out2;  // out2: second output of the generic key-range rounds
  gpu::DeviceBuffer fetched;  // device fetch: bytes of the partitions the providers declined as descriptors
  gpu::GenericMerger merger;
  gpu::DeviceBlockDecoder decoder;
  gpu::PinnedBuffer ring;          // 2 x kPieceBytes, D2H staging of merged output
  gpu::GenericRoundsWs rounds;     // key-range round planner scratch (device fetch, generic keys)
  gpu::DeviceBuffer frame_scratch, frame_descs; // device framing walk of compressed partitions (device fetch)
  hipEvent_t piece_ev[2] = {nullptr, nullptr};
  // SDMA delivery ring of stream_out: kOutSlots pieces of kOutPiece bytes on the GPU's NUMA node, each
  // with its completion signal
  gpu::SdmaEngine* oeng = nullptr;
  uint8_t* oring = nullptr;
  std::vector<hsa_signal_t> osig;
  bool sdma_out_ok = true;
  int out_ways = 1;  // SDMA engines each delivery piece is split over (the job's long pole: more)
  hsa_signal_t h2d_sig{};    // SDMA copies of this workspace: H2D of pinned spans (device_merge), LPQ spill D2H
  bool h2d_sdma_ok = true;
  double h2d_ms = 0, device_ms = 0, d2h_ms = 0, sink_ms = 0;
  ~DeviceWorkspace() {
    for (auto sg : osig) {
      try {
        gpu::SdmaEngine::wait(sg);  // a copy still in flight lands before the ring is reused
      } catch (...) {
      }
      oeng->destroy_signal(sg);
    }
    if (oring) oeng->release_ring(oring, (size_t)kOutSlots * kOutPiece);
    if (h2d_sig.handle) {
      try {
        gpu::SdmaEngine::wait(h2d_sig);
      } catch (...) {
      }
      (void)hsa_signal_destroy(h2d_sig);
    }
    for (auto e : piece_ev)
      if (e) (void)hipEventDestroy(e);
    if (cs) (void)hipStreamDestroy(cs);
  }
  void reset_stats() {
    h2d_ms = device_ms = d2h_ms = sink_ms = 0;
    out_ways = 1;
  }
  // D2H stream of streamed deliveries (the merge stream is busy with the next round)
  hipStream_t copy_stream() {
    if (!cs) HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    return cs;
  }
  hipStream_t cs = nullptr;
  static void ensure(gpu::DeviceBuffer& b, int64_t bytes) {
    bytes = std::max<int64_t>(bytes, 16);
    if ((int64_t)b.size() < bytes) b.alloc_local((size_t)(bytes + bytes / 8));
  }
  int64_t device_bytes() const {
    return (int64_t)(in.held() + out.held() + packed.held() + out2.held() + fetched.held() + frame_scratch.held() +
                     frame_descs.held()) +
           merger.workspace_bytes();
  }
};

// a task's stream from the device's pool (gpu::pooled_stream), handed back when the task is done
struct StreamGuard {
  hipStream_t s = nullptr;
  ~StreamGuard() { gpu::return_stream(s); }
};

// Merge host-resident runs on the device. `codec` != kNone: the runs are block-compressed streams
// decoded in HBM (falls back to a host decode when the framing needs it).
// Host spans of the runs to merge (pinned when they come from the arenas).
struct Span {
  const uint8_t* p;
  int64_t len;
  const uint8_t* dev = nullptr;  // device copy staged while the fetch went on (EarlyStager)
};

// Stages fetched partitions to HBM as soon as each one is complete in pinned memory, so the H2D
// copies overlap the remaining fetches (one issuing thread, one copy stream: the round-1 attempt
// issued from every drain thread and the copies contended). Device memory comes from a bump
// arena of 256 MiB blocks (a partition never straddles blocks); reset() recycles it once the
// group's merge has finished.
class EarlyStager {
 public:
  // SDMA (default, UDA_EARLY_H2D_SDMA=0 for hipMemcpyAsync): the copies run on a copy engine. A
  // hipMemcpyAsync H2D from pinned memory runs as a blit kernel whose host reads slowed the
  // concurrent fetch memcpys into the same arena about 8x when partitions were staged piecewise.
  explicit EarlyStager(int device) : device_(device) {
    s_ = gpu::pooled_stream();
    const char* e = std::getenv("UDA_EARLY_H2D_SDMA");
    if (!e || std::atoi(e) != 0) {
      try {
        sdma_ = &gpu::SdmaEngine::for_device(device);
        sig_ = sdma_->make_signal();
        gpu::SdmaEngine::arm(sig_, 0);
        for (auto& g : gsig_) {
          g = sdma_->make_signal();
          gpu::SdmaEngine::arm(g, 0);
        }
      } catch (const std::exception& ex) {
        UDA_LOG(kWarn, "early staging: no SDMA engine (%s); using hipMemcpyAsync", ex.what());
        sdma_ = nullptr;
      }
    }
    thr_ = std::thread([this] { loop(); });
  }
  ~EarlyStager() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    thr_.join();
    (void)hipStreamSynchronize(s_);
    gpu::return_stream(s_);
    if (sdma_) {
      std::vector<hsa_signal_t> all{sig_};
      all.insert(all.end(), gsig_, gsig_ + kGroups);
      for (hsa_signal_t g : all) {
        try {
          gpu::SdmaEngine::wait(g);
        } catch (...) {
        }
        sdma_->destroy_signal(g);
      }
    }
  }
  const char* engine() const { return sdma_ ? "sdma" : "hip"; }
  // Device address the partition will be copied to; the copy is issued asynchronously.
  const uint8_t* submit(const uint8_t* host, int64_t len) {
    uint8_t* d = reserve(len);
    copy(host, d, len);
    return d;
  }
  // A partition's device span, filled piecewise by copy() as its bytes land in pinned memory.
  uint8_t* reserve(int64_t len) {
    std::lock_guard<std::mutex> g(mu_);
    return alloc(len);
  }
  // group >= 0 (SDMA only): the copy also counts toward flush_group(group), so a caller can wait for
  // one batch of copies (a progressive merge's phase) while later batches are still being queued.
  void copy(const uint8_t* host, uint8_t* dev, int64_t len, int group = -1) {
    if (len <= 0) return;
    std::lock_guard<std::mutex> g(mu_);
    if (group >= kGroups || (group >= 0 && !sdma_)) throw UdaError("early staging: bad copy group");
    if (group >= 0) ++gqueued_[group];
    q_.push_back(Job{host, dev, len, trace::host_enabled() ? trace::now_ns() : 0, group});
    cv_.notify_all();
  }
  static constexpr int kGroups = 16;
  bool sdma() const { return sdma_ != nullptr; }
  // Every copy of `group` queued so far has completed.
  void flush_group(int group) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return gqueued_[group] == 0 || !error_.empty(); });
    if (!error_.empty()) throw UdaError("early H2D staging failed: " + error_);
    lk.unlock();
    try {
      gpu::SdmaEngine::wait(gsig_[group]);
    } catch (const std::exception& ex) {
      gpu::SdmaEngine::arm(gsig_[group], 0);
      throw UdaError(std::string("early H2D staging failed: ") + ex.what());
    }
  }
  // Every submitted copy has completed.
  void flush() {
    const int64_t tf = trace::host_enabled() ? trace::now_ns() : 0;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return q_.empty() && busy_ == 0; });
    lk.unlock();
    HIP_CHECK(hipStreamSynchronize(s_));
    if (sdma_) {
      for (int g = -1; g < kGroups; ++g) {
        hsa_signal_t sg = g < 0 ? sig_ : gsig_[g];
        try {
          gpu::SdmaEngine::wait(sg);
        } catch (const std::exception& ex) {
          gpu::SdmaEngine::arm(sg, 0);
          throw UdaError(std::string("early H2D staging failed: ") + ex.what());
        }
      }
    }
    if (!error_.empty()) throw UdaError("early H2D staging failed: " + error_);
    if (tf) trace::host_event("stage_flush", bytes_, copies_, tf, trace::now_ns());
  }
  void reset() {
    flush();
    std::lock_guard<std::mutex> g(mu_);
    for (auto& b : blocks_) b.used = 0;
    cur_ = 0;
    issue_ms_ = 0;
    copies_ = 0;
    bytes_ = 0;
  }
  // reset() and give the device blocks back (a task switching to direct RPQ rounds: its staged copies
  // are not used, and the rounds' workspaces need that HBM within the budget)
  void release_blocks() {
    reset();
    std::lock_guard<std::mutex> g(mu_);
    blocks_.clear();
  }
  double issue_ms() const { return issue_ms_; }
  int64_t copies() const { return copies_; }
  int64_t bytes() const { return bytes_; }
  int64_t device_bytes() {
    std::lock_guard<std::mutex> g(mu_);
    int64_t n = 0;
    for (const auto& b : blocks_) n += (int64_t)b.buf.held();
    return n;
  }

 private:
  struct Job {
    const uint8_t* host;
    uint8_t* dev;
    int64_t len;
    int64_t t_enq;  // trace: when the copy was queued
    int group;
  };
  struct Block {
    gpu::DeviceBuffer buf;
    int64_t used = 0;
  };
  uint8_t* alloc(int64_t len) {  // mu_ held
    len = (std::max<int64_t>(len, 1) + 255) & ~(int64_t)255;
    for (; cur_ < blocks_.size(); ++cur_)
      if ((int64_t)blocks_[cur_].buf.size() - blocks_[cur_].used >= len) break;
    if (cur_ == blocks_.size()) {
      blocks_.emplace_back();
      HIP_CHECK(hipSetDevice(device_));
      blocks_.back().buf.alloc((size_t)std::max<int64_t>(len, 256ll << 20));
    }
    Block& b = blocks_[cur_];
    uint8_t* p = b.buf.as<uint8_t>() + b.used;
    b.used += len;
    return p;
  }
  void loop() {
    (void)hipSetDevice(device_);
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        j = q_.front();
        q_.pop_front();
        ++busy_;
      }
      const auto t0 = std::chrono::steady_clock::now();
      std::string err;
      if (sdma_) {
        hsa_signal_t sg = j.group >= 0 ? gsig_[j.group] : sig_;
        gpu::SdmaEngine::add(sg, 1);
        try {
          sdma_->copy_h2d(j.dev, j.host, (size_t)j.len, sg);
        } catch (const std::exception& ex) {
          gpu::SdmaEngine::add(sg, -1);
          err = ex.what();
        }
      } else {
        const hipError_t e = hipMemcpyAsync(j.dev, j.host, (size_t)j.len, hipMemcpyHostToDevice, s_);
        if (e != hipSuccess) err = hipGetErrorString(e);
      }
      issue_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (j.t_enq) {
        trace::host_event("stage_wait", j.len, (int64_t)(uintptr_t)j.host, j.t_enq, trace::now_ns());
      }
      std::lock_guard<std::mutex> g(mu_);
      if (!err.empty() && error_.empty()) error_ = err;
      bytes_ += j.len;
      ++copies_;
      --busy_;
      if (j.group >= 0) --gqueued_[j.group];  // issued (its signal tracks completion)
      cv_.notify_all();
    }
  }
  int device_;
  hipStream_t s_ = nullptr;
  gpu::SdmaEngine* sdma_ = nullptr;
  hsa_signal_t sig_{};  // outstanding SDMA copies
  hsa_signal_t gsig_[kGroups]{};  // outstanding copies per group
  int64_t gqueued_[kGroups]{};    // queued, not yet issued, per group
  std::thread thr_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  int busy_ = 0;
  bool stop_ = false;
  std::string error_;
  std::vector<Block> blocks_;
  size_t cur_ = 0;
  double issue_ms_ = 0;
  int64_t copies_ = 0;
  int64_t bytes_ = 0;
};

// Process-wide cache of the per-device objects a GPU reduce task builds (HBM workspaces, the
// pinned D2H ring, the early-staging arena and its copy thread): one reducer process runs many
// reduce tasks in sequence, and building these costs tens of ms per task (pinning a 128 MiB ring,
// hipMalloc of GBs, hipFree synchronizing the device). An object goes back to the cache only
// after a task that used it ended cleanly.
template <class T>
class DevicePool {
 public:
  static DevicePool& get() {
    static DevicePool* p = [] {
      auto* q = new DevicePool;  // never destroyed: HIP may be torn down first at exit
      // idle objects hold HBM: the device's byte budget trims them (largest first) under pressure
      gpu::HbmLedger::get().add_pool({[q](int d, int64_t want) { return q->trim(d, want); },
                                      [q](int d) { return q->idle(d); }});
      return q;
    }();
    return *p;
  }
  template <class Make>
  std::unique_ptr<T> acquire(int device, Make&& make) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = idle_[device];
      if (!v.empty()) {
        std::unique_ptr<T> o = std::move(v.back());
        v.pop_back();
        return o;
      }
    }
    return make();
  }
  // The idle object last used by the task most like this one: the closest pool_key (the input bytes of
  // the task that used it; ties to the larger object), then tagged with `key`. The jobs of a wave repeat
  // their shapes, so a skewed task gets back the workspace it grew before. Handing it a small one makes
  // it grow again (and hipFree the old buffers, which synchronizes the device under every other task),
  // and what its size promises is no guide: tasks of any input size beyond one round size their
  // workspaces to the round (config #5, 100 GB: 16.6 GB/s last-in, 20-30 by size, see BENCHMARKS.md).
  template <class Make>
  std::unique_ptr<T> acquire_fit(int device, int64_t key, Make&& make) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = idle_[device];
      if (!v.empty()) {
        size_t best = 0;
        for (size_t i = 1; i < v.size(); ++i) {
          const int64_t b = v[best]->pool_key, c = v[i]->pool_key;
          const int64_t db = b > key ? b - key : key - b, dc = c > key ? c - key : key - c;
          if (dc < db || (dc == db && v[i]->device_bytes() > v[best]->device_bytes())) best = i;
        }
        std::unique_ptr<T> o = std::move(v[best]);
        v.erase(v.begin() + (long)best);
        o->pool_key = key;
        return o;
      }
    }
    std::unique_ptr<T> o = make();
    o->pool_key = key;
    return o;
  }
  void release(int device, std::unique_ptr<T> o) {
    std::lock_guard<std::mutex> g(mu_);
    auto& v = idle_[device];
    if (v.size() < kMaxIdle) v.push_back(std::move(o));
  }
  int64_t trim(int device, int64_t want) {
    std::vector<std::unique_ptr<T>> drop;
    int64_t got = 0;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = idle_[device];
      std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a->device_bytes() < b->device_bytes(); });
      while (!v.empty() && got < want) {
        got += v.back()->device_bytes();
        drop.push_back(std::move(v.back()));
        v.pop_back();
      }
    }
    if (!drop.empty()) {
      int cur = 0;
      HIP_CHECK(hipGetDevice(&cur));
      HIP_CHECK(hipSetDevice(device));
      drop.clear();
      HIP_CHECK(hipSetDevice(cur));
    }
    return got;
  }
  int64_t idle(int device) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t n = 0;
    for (auto& o : idle_[device]) n += o->device_bytes();
    return n;
  }

 private:
  // Idle objects are bounded in bytes by the device's HBM budget (trimmed under pressure); the count
  // bound only limits the host memory they pin (a workspace's D2H ring is 128 MiB of pinned DRAM).
  // 16 concurrent reduce tasks per GPU (the bench shape) must find their workspaces again: a dropped
  // one is freed, and hipFree synchronizes the whole device under the other tasks.
  static constexpr size_t kMaxIdle = 32;
  std::mutex mu_;
  std::map<int, std::vector<std::unique_ptr<T>>> idle_;
};

template <class T>
struct PoolLease {
  int device;
  std::unique_ptr<T> obj;
  bool clean = false;  // set when the task ended without an error
  ~PoolLease() {
    if (obj && clean) DevicePool<T>::get().release(device, std::move(obj));
  }
};

// Admission of staged GPU reduce tasks per device (mapred.uda.gpu.max.concurrent.merges, default 0 =
// no limit).
// Reduce tasks started together run their phases in lockstep: all fetch and copy to HBM at once (the
// H2D direction of PCIe busy, D2H idle), then all merge, then all deliver (D2H busy, H2D idle). With
// at most `cap` tasks admitted, in arrival order, a task's fetch and H2D overlap the merge and D2H of
// the tasks ahead of it, so both PCIe directions stay busy. Tasks wait in FIFO order of arrival.
class DeviceGate {
 public:
  // gate 0: staged GPU merges (mapred.uda.gpu.max.concurrent.merges); gate 1: device block decodes
  // of compressed descriptor tasks (mapred.uda.gpu.decode.slots)
  // gate 2: declined-partition byte fetches of device-fetch tasks (mapred.uda.gpu.fetch.bytes.slots)
  static DeviceGate& get(int which = 0) {
    // never destroyed: tasks may outlive static teardown
    static DeviceGate* g[3] = {new DeviceGate, new DeviceGate, new DeviceGate};
    return *g[(unsigned)which % 3];
  }
  // false if `stopped` became true while waiting
  template <class Stop>
  bool acquire(int device, int cap, Stop&& stopped) {
    std::unique_lock<std::mutex> lk(mu_);
    Dev& d = devs_[device];
    const uint64_t me = d.next_ticket++;
    d.waiting.push_back(me);
    for (;;) {
      if (d.used < cap && d.waiting.front() == me) {
        d.waiting.pop_front();
        ++d.used;
        cv_.notify_all();
        return true;
      }
      if (stopped()) {
        d.waiting.erase(std::find(d.waiting.begin(), d.waiting.end(), me));
        cv_.notify_all();
        return false;
      }
      cv_.wait_for(lk, std::chrono::milliseconds(20));
    }
  }
  void release(int device) {
    std::lock_guard<std::mutex> g(mu_);
    --devs_[device].used;
    cv_.notify_all();
  }
  // host function enqueued behind a gated copy: frees the slot the moment the copy has landed (not when
  // the task comes back for it after consuming the previous piece)
  static void release_cb(void* device) { get().release((int)(intptr_t)device); }

 private:
  struct Dev {
    int used = 0;
    uint64_t next_ticket = 0;
    std::deque<uint64_t> waiting;
  };
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int, Dev> devs_;
};

// Staged GPU merges running per device (the progressive-phase default asks whether a task is alone).
std::atomic<int>& staged_merges(int device) {
  static std::atomic<int> n[64];
  return n[device & 63];
}
struct StagedCount {
  int device;
  explicit StagedCount(int d) : device(d) { staged_merges(device).fetch_add(1); }
  ~StagedCount() { staged_merges(device).fetch_sub(1); }
};

struct GateLease {
  int device = -1;
  int which = 0;
  ~GateLease() {
    if (device >= 0) DeviceGate::get(which).release(device);
  }
};

// on_round: deliver the merged output in key-range rounds while the device merges the next one
// (GenericMerger::merge); time spent in it is not counted as device time.
// pinned_src: the host spans are pinned (spill arenas): their H2D goes to an SDMA engine (not the
// delivery engine) instead of a blit kernel whose host reads would slow the merge kernels beside it.
DeviceMergeOut device_merge(DeviceWorkspace& ws, const std::vector<Span>& in_runs, Codec codec, KeyKind kind,
                            int64_t spacing, hipStream_t s, const gpu::GenericMerger::RoundFn& on_round = nullptr,
                            bool pinned_src = false) {
  double round_ms = 0;
  gpu::GenericMerger::RoundFn timed;
  if (on_round)
    timed = [&](const std::vector<int64_t>& cuts, int64_t records, bool last) {
      const auto tr = std::chrono::steady_clock::now();
      on_round(cuts, records, last);
      round_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
    };
  auto t0 = std::chrono::steady_clock::now();
  std::vector<const uint8_t*> ptrs;
  std::vector<int64_t> lens;
  bool all_staged = codec == Codec::kNone && !in_runs.empty();
  for (const Span& sp : in_runs) {
    ptrs.push_back(sp.p);
    lens.push_back(sp.len);
    all_staged = all_staged && sp.dev != nullptr;
  }
  if (all_staged) {  // the partitions reached HBM while the fetch went on
    int64_t total = 0;
    std::vector<const uint8_t*> runs;
    for (const Span& sp : in_runs) {
      runs.push_back(sp.dev);
      total += sp.len;
    }
    DeviceWorkspace::ensure(ws.out, total);
    auto t1 = std::chrono::steady_clock::now();
    ws.h2d_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    gpu::GenericMergeResult r =
        ws.merger.merge(runs, lens, (int)kind, ws.out.as<uint8_t>(), total, spacing, s, timed);
    HIP_CHECK(hipStreamSynchronize(s));
    ws.device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count() - round_ms;
    DeviceMergeOut res;
    res.bytes = r.bytes;
    res.cuts = std::move(r.cuts);
    res.records = r.records;
    return res;
  }
  gpu::BlockPlan plan;
  bool decode_on_device = false;
  std::vector<std::vector<uint8_t>> host_raw;  // host-decoded fallback
  if (codec != Codec::kNone) {
    decode_on_device = gpu::plan_block_streams(codec, ptrs, lens, &plan);
    if (!decode_on_device) {
      UDA_LOG(kInfo, "device decode: framing needs a host decode (multi-chunk %s block)", codec_name(codec));
      for (size_t i = 0; i < ptrs.size(); ++i) {
        BlockDecoder dec(codec);
        dec.feed(ptrs[i], (size_t)lens[i]);
        std::vector<uint8_t> raw, buf(1 << 20);
        for (size_t n; (n = dec.read(buf.data(), buf.size())) > 0;) raw.insert(raw.end(), buf.begin(), buf.begin() + (long)n);
        if (!dec.idle()) throw UdaError("truncated compressed partition");
        host_raw.push_back(std::move(raw));
      }
      ptrs.clear();
      lens.clear();
      for (auto& r : host_raw) {
        ptrs.push_back(r.data());
        lens.push_back((int64_t)r.size());
      }
    }
  }
  int64_t staged = 0;
  for (auto l : lens) staged += l;
  const int64_t total = decode_on_device ? plan.raw_total : staged;
  DeviceWorkspace::ensure(ws.in, total);
  DeviceWorkspace::ensure(ws.out, total);
  if (decode_on_device) DeviceWorkspace::ensure(ws.packed, staged);
  gpu::DeviceBuffer& in = ws.in;
  gpu::DeviceBuffer& out = ws.out;
  uint8_t* stage = decode_on_device ? ws.packed.as<uint8_t>() : in.as<uint8_t>();
  std::vector<const uint8_t*> runs;
  std::vector<int64_t> bytes;
  int64_t off = 0;
  gpu::SdmaEngine* h2d = nullptr;
  if (pinned_src && host_raw.empty() && ws.h2d_sdma_ok) {
    try {
      int dev = 0;
      HIP_CHECK(hipGetDevice(&dev));
      h2d = &gpu::SdmaEngine::for_device(dev);
      if (!ws.h2d_sig.handle) ws.h2d_sig = h2d->make_signal();
      gpu::SdmaEngine::arm(ws.h2d_sig, 0);
    } catch (const std::exception&) {
      h2d = nullptr;
      ws.h2d_sdma_ok = false;
    }
  }
  for (size_t i = 0; i < ptrs.size(); ++i) {
    if (lens[i] > 0 && h2d) {
      gpu::SdmaEngine::add(ws.h2d_sig, 1);
      h2d->copy_h2d(stage + off, ptrs[i], (size_t)lens[i], ws.h2d_sig);
    } else if (lens[i] > 0) {
      HIP_CHECK(hipMemcpyAsync(stage + off, ptrs[i], (size_t)lens[i], hipMemcpyHostToDevice, s));
    }
    if (decode_on_device) {
      runs.push_back(in.as<uint8_t>() + plan.raw_offset[i]);
      bytes.push_back(plan.raw_offset[i + 1] - plan.raw_offset[i]);
    } else {
      runs.push_back(in.as<uint8_t>() + off);
      bytes.push_back(lens[i]);
    }
    off += lens[i];
  }
  if (h2d) gpu::SdmaEngine::wait(ws.h2d_sig);
  HIP_CHECK(hipStreamSynchronize(s));
  auto t1 = std::chrono::steady_clock::now();
  ws.h2d_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  const int64_t tm = trace::host_enabled() ? trace::now_ns() : 0;
  if (tm) trace::host_event("dm_h2d", staged, (int64_t)ptrs.size(), tm - (int64_t)((t1 - t0).count()), tm);
  DeviceMergeOut res;
  if (decode_on_device) {
    ws.decoder.decode(codec, plan, ws.packed.as<uint8_t>(), in.as<uint8_t>(), s);
    res.decoded_blocks = (int64_t)plan.descs.size();
  }
  host_raw.clear();
  gpu::GenericMergeResult r = ws.merger.merge(runs, bytes, (int)kind, out.as<uint8_t>(), total, spacing, s, timed);
  HIP_CHECK(hipStreamSynchronize(s));
  ws.device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count() - round_ms;
  if (tm) trace::host_event("dm_merge", total, (int64_t)ptrs.size(), tm, trace::now_ns());
  res.bytes = r.bytes;
  res.cuts = std::move(r.cuts);
  res.records = r.records;
  return res;
}

// piece boundaries (in cut indices) of a merged output: pieces of up to `limit` bytes ending on record
// boundaries; empty if a single cut interval is larger than `limit`
std::vector<size_t> piece_bounds(const std::vector<int64_t>& cuts, int64_t limit) {
  const size_t nb = cuts.size() - 1;
  std::vector<size_t> pb{0};
  while (pb.back() < nb) {
    const size_t j = pb.back();
    if (cuts[j + 1] - cuts[j] > limit) return {};
    size_t k = j + 1;
    while (k < nb && cuts[k + 1] - cuts[j] <= limit) ++k;
    pb.push_back(k);
  }
  return pb;
}

// Stream the merged output of `m` (in ws.out, complete on the device) to the host in pieces that end on
// record boundaries (the cuts): up to kOutSlots pieces of kOutPiece bytes queued on the GPU's SDMA
// engines ahead of the consumer, fn(piece k) running while pieces k+1.. land. fn(ptr, first_cut,
// last_cut) gets the bytes of cuts [first_cut, last_cut] (ptr = byte cuts[first_cut]). A record larger
// than a piece, or no SDMA engine: two 64 MiB pieces through hipMemcpyAsync on `s`.
template <typename Fn>
void stream_out(DeviceWorkspace& ws, const DeviceMergeOut& m, hipStream_t s, Fn&& fn, const uint8_t* src = nullptr) {
  const size_t nb = m.cuts.size() < 2 ? 0 : m.cuts.size() - 1;
  if (nb == 0) return;
  const uint8_t* out = src ? src : ws.out.as<uint8_t>();
  if (ws.sdma_out_ok && !ws.oring) {
    try {
      int dev = 0;
      HIP_CHECK(hipGetDevice(&dev));
      ws.oeng = &gpu::SdmaEngine::for_device(dev);
      ws.oring = static_cast<uint8_t*>(ws.oeng->acquire_ring((size_t)kOutSlots * kOutPiece));
      for (int i = 0; i < kOutSlots; ++i) ws.osig.push_back(ws.oeng->make_signal());
    } catch (const std::exception& e) {
      UDA_LOG(kInfo, "stream_out: no SDMA delivery ring (%s): hipMemcpyAsync pieces", e.what());
      ws.sdma_out_ok = false;
    }
  }
  if (ws.oring) {
    const std::vector<size_t> pb = piece_bounds(m.cuts, kOutPiece);
    if (!pb.empty()) {
      const size_t np = pb.size() - 1;
      gpu::SdmaEngine& eng = *ws.oeng;
      auto issue = [&](size_t k) {
        const int64_t b = m.cuts[pb[k]], len = m.cuts[pb[k + 1]] - b;
        hsa_signal_t sg = ws.osig[k % kOutSlots];
        gpu::SdmaEngine::arm(sg, eng.parts((size_t)len, ws.out_ways));
        eng.copy_d2h(ws.oring + (k % kOutSlots) * kOutPiece, out + b, (size_t)len, sg, ws.out_ways);
      };
      size_t issued = 0, k = 0;
      // a consumer that throws (a stopped task) leaves copies in flight into the ring: they land before
      // the ring and its signals serve the next output
      struct Drain {
        DeviceWorkspace& ws;
        size_t& issued;
        size_t& k;
        ~Drain() {
          for (size_t j = k; j < issued; ++j) {
            try {
              gpu::SdmaEngine::wait(ws.osig[j % kOutSlots]);
            } catch (...) {
            }
          }
        }
      } drain{ws, issued, k};
      for (; issued < std::min<size_t>(np, kOutSlots); ++issued) issue(issued);
      for (; k < np; ++k) {
        auto t0 = std::chrono::steady_clock::now();
        gpu::SdmaEngine::wait(ws.osig[k % kOutSlots]);
        auto t1 = std::chrono::steady_clock::now();
        ws.d2h_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
        const int64_t tp = trace::host_enabled() ? trace::now_ns() : 0;
        if (tp) trace::host_event("so_wait", (int64_t)(uintptr_t)&ws, 0, tp - (int64_t)(t1 - t0).count(), tp);
        fn(ws.oring + (k % kOutSlots) * kOutPiece, pb[k], pb[k + 1]);
        ws.sink_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
        if (tp) trace::host_event("so_sink", (int64_t)(uintptr_t)&ws, m.cuts[pb[k + 1]] - m.cuts[pb[k]], tp,
                                  trace::now_ns());
        if (k + kOutSlots < np) issue(issued++);  // its slot was just consumed
      }
      return;
    }
  }
  if (ws.ring.size() < (size_t)(2 * kPieceBytes)) {  // on the GPU's NUMA node, like the consumer copying out of it
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    ws.ring.alloc_on_node((size_t)(2 * kPieceBytes), gpu::device_numa_node(dev));
  }
  for (auto& e : ws.piece_ev)
    if (!e) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // piece boundaries in cut indices
  std::vector<size_t> pb{0};
  while (pb.back() < nb) {
    size_t j = pb.back();
    const int64_t start = m.cuts[j];
    size_t k = j + 1;
    while (k < nb && m.cuts[k + 1] - start <= kPieceBytes) ++k;
    pb.push_back(k);
  }
  auto enqueue = [&](size_t piece) {
    const int slot = (int)(piece & 1);
    const int64_t b = m.cuts[pb[piece]], e = m.cuts[pb[piece + 1]];
    if (e - b > kPieceBytes) throw UdaError("record larger than the D2H piece");
    HIP_CHECK(hipMemcpyAsync(ws.ring.as<uint8_t>() + slot * kPieceBytes, out + b, (size_t)(e - b),
                             hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(ws.piece_ev[slot], s));
  };
  const size_t np = pb.size() - 1;
  enqueue(0);
  for (size_t piece = 0; piece < np; ++piece) {
    const int slot = (int)(piece & 1);
    auto t0 = std::chrono::steady_clock::now();
    HIP_CHECK(hipEventSynchronize(ws.piece_ev[slot]));
    auto t1 = std::chrono::steady_clock::now();
    ws.d2h_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    const int64_t tp = trace::host_enabled() ? trace::now_ns() : 0;
    if (tp) trace::host_event("so_wait", (int64_t)(uintptr_t)&ws, 0, tp - (int64_t)(t1 - t0).count(), tp);
    if (piece + 1 < np) enqueue(piece + 1);
    fn(ws.ring.as<uint8_t>() + slot * kPieceBytes, pb[piece], pb[piece + 1]);
    ws.sink_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    if (tp) trace::host_event("so_sink", (int64_t)(uintptr_t)&ws, m.cuts[pb[piece + 1]] - m.cuts[pb[piece]], tp,
                              trace::now_ns());
  }
}

std::string key_at(const uint8_t* p, int64_t avail) {
  RecordView rv;
  if (ifile_parse(p, (size_t)avail, &rv) != Parse::kRecord) throw UdaError("spill index: bad record boundary");
  return std::string(reinterpret_cast<const char*>(rv.key), (size_t)rv.klen);
}

int cmp_key(KeyKind kind, const std::string& a, const std::string& b) {
  return key_compare(kind, reinterpret_cast<const uint8_t*>(a.data()), (int)a.size(),
                     reinterpret_cast<const uint8_t*>(b.data()), (int)b.size());
}

// Direct RPQ (see merge_gpu): a fetched partition, already a sorted run in pinned DRAM, becomes an RPQ
// input as it is: the record boundary at or after every `spacing` bytes and its key, by one walk of
// the VInt headers. bytes = the records (an EOF marker ends the walk and is left out).
SpillRun index_host_run(uint8_t* p, int64_t len, int64_t spacing) {
  const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
  SpillRun run;
  run.mem = p;
  int64_t off = 0, next_cut = 0;
  while (off < len) {
    // between cuts: skip records with one-byte VInt headers (lengths < 128) without parsing them
    while (off < next_cut && off + 2 <= len) {
      const int8_t k1 = (int8_t)p[off], v1 = (int8_t)p[off + 1];
      if ((k1 | v1) < 0) break;  // multi-byte header or the EOF marker: the parser below
      const int64_t nx = off + 2 + k1 + v1;
      if (nx > len) break;  // truncated: the parser below reports it
      off = nx;
    }
    if (off >= len) break;
    RecordView rv;
    const Parse ps = ifile_parse(p + off, (size_t)(len - off), &rv);
    if (ps == Parse::kEof) break;
    if (ps != Parse::kRecord) throw UdaError("hybrid index: bad record in a fetched partition");
    if (off >= next_cut) {
      run.cut.push_back(off);
      run.key.emplace_back(reinterpret_cast<const char*>(rv.key), (size_t)rv.klen);
      next_cut = off + spacing;
    }
    off += rv.size();
  }
  run.bytes = off;
  if (tt) trace::host_event("index", len, (int64_t)run.cut.size(), tt, trace::now_ns());
  return run;
}

// index_host_run for a partition that lands in byte phases: walks the complete records of [pos, limit)
// (the bytes landed so far), a sample every `spacing` bytes; a record the landed bytes cut is left for
// the next call. Samples go to the caller's vectors; the cursor and the last complete record stay here.
struct RunCursor {
  int64_t pos = 0, next_cut = 0;
  int64_t last = -1;  // start of the last complete record walked
  bool eof = false;
  void advance(const uint8_t* p, int64_t limit, int64_t spacing, std::vector<int64_t>* cut, std::vector<std::string>* key) {
    while (!eof && pos < limit) {
      while (pos < next_cut && pos + 2 <= limit) {  // one-byte VInt headers: skip without parsing
        const int8_t k1 = (int8_t)p[pos], v1 = (int8_t)p[pos + 1];
        if ((k1 | v1) < 0) break;
        const int64_t nx = pos + 2 + k1 + v1;
        if (nx > limit) break;
        last = pos;
        pos = nx;
      }
      if (pos >= limit) break;
      RecordView rv;
      const Parse ps = ifile_parse(p + pos, (size_t)(limit - pos), &rv);
      if (ps == Parse::kEof) {
        eof = true;
        break;
      }
      if (ps == Parse::kPartial) break;  // the rest of it lands with a later phase
      if (ps != Parse::kRecord) throw UdaError("hybrid index: bad record in a fetched partition");
      if (pos >= next_cut) {
        cut->push_back(pos);
        key->emplace_back(reinterpret_cast<const char*>(rv.key), (size_t)rv.klen);
        next_cut = pos + spacing;
      }
      last = pos;
      pos += rv.size();
    }
  }
  std::string last_key(const uint8_t* p) const {
    RecordView rv;
    if (last < 0 || ifile_parse(p + last, (size_t)(pos - last), &rv) != Parse::kRecord) return std::string();
    return std::string(reinterpret_cast<const char*>(rv.key), (size_t)rv.klen);
  }
};

}  // namespace

void ReduceTask::release_descriptors(const std::set<std::string>& hosts, const std::string& holder) {
  if (hosts.empty() || !transport_) return;
  struct Wait {  // outlives this call if a provider answers late
    std::mutex m;
    std::condition_variable c;
    size_t left = 0;
  };
  auto w = std::make_shared<Wait>();
  w->left = hosts.size();
  for (const auto& h : hosts) {
    FetchRequest req;
    req.job_id = init_.job_id;
    req.map_id = "*";
    req.reduce_id = 0;
    req.buf_len = kDescriptorRelease;
    req.holder = holder;
    fetch_begin();
    transport_->fetch(h, req, nullptr, [this, w](const FetchAck&) {
      {
        std::lock_guard<std::mutex> g(w->m);
        --w->left;
        w->c.notify_all();
      }
      fetch_end();
    });
  }
  std::unique_lock<std::mutex> lk(w->m);
  // a provider that does not answer keeps the references until its backstop drops them
  if (!w->c.wait_for(lk, std::chrono::seconds(10), [&] { return w->left == 0; }))
    throw UdaError("descriptor release not acknowledged by " + std::to_string(w->left) + " provider(s)");
}

namespace {
// once per process: the context and the library's code objects (loaded at the first kernel launch);
// later prewarms must not hipFree (it synchronizes the device under running tasks)
void warm_code(int device) {
  static std::once_flag code_once;
  std::call_once(code_once, [device] {
    uint8_t* tmp = nullptr;  // raw hipMalloc: the prewarm is not the merge (fault injection hits the merge)
    HIP_CHECK(hipMalloc(&tmp, 4096));
    HIP_CHECK(hipMemsetAsync(tmp, 0, 64, nullptr));
    gpu::launch_max_i32(reinterpret_cast<int32_t*>(tmp), 1, reinterpret_cast<unsigned int*>(tmp + 32), nullptr);
    HIP_CHECK(hipStreamSynchronize(nullptr));
    try {  // the SDMA engines' queues (staging H2D, delivery D2H)
      gpu::SdmaEngine::for_device(device).warm(tmp);
    } catch (const std::exception& e) {
      UDA_LOG(kWarn, "GPU prewarm: SDMA warm-up: %s", e.what());
    }
    HIP_CHECK(hipFree(tmp));
  });
}

// `n` pooled merge workspaces with their pinned D2H rings (NUMA-local), held at once so the pool keeps n
void warm_workspaces(int device, int n) {
  std::vector<std::unique_ptr<PoolLease<DeviceWorkspace>>> held;
  for (int i = 0; i < std::max(1, n); ++i) {
    held.emplace_back(new PoolLease<DeviceWorkspace>{
        device, DevicePool<DeviceWorkspace>::get().acquire(device, [] { return std::make_unique<DeviceWorkspace>(); })});
    auto& wl = *held.back();
    if (wl.obj->ring.size() < (size_t)(2 * kPieceBytes))
      wl.obj->ring.alloc_on_node((size_t)(2 * kPieceBytes), gpu::device_numa_node(device));
    wl.clean = true;
  }
}
}  // namespace

void prewarm_node_merges(int device, int tasks, int64_t round_bytes, int maps, int64_t kv_buf) {
  HIP_CHECK(hipSetDevice(device));
  (void)gpu::SdmaEngine::for_device(device);
  warm_code(device);
  warm_workspaces(device, tasks);
  gpu::prewarm_streams(device, tasks);
  gpu::DeviceReduceConfig cfg;
  cfg.device = device;
  cfg.kv_buf_bytes = kv_buf;
  cfg.round_bytes = round_bytes;
  gpu::prewarm_device_reduce(cfg, std::max(1, maps), tasks);
}

// Every reduce task of a Hadoop job usually runs in a fresh JVM (YarnChild), so what a warm process
// keeps in its pools (HIP context, code objects, pinned rings and arenas, workspaces) a task would build
// on its critical path: a 2 GB task went 27 -> 3.9 GB/s cold (profiles/r3_netmerger2.json). INIT comes
// while most maps still run (reduce slow-start), so the task builds them then. Best effort: any failure
// leaves the merge to build what it needs as before.
void ReduceTask::prewarm_gpu(PrewarmConf pc) {
  const auto t0 = std::chrono::steady_clock::now();
  auto tp = t0;
  std::string phases;
  auto lap = [&](const char* name) {
    const auto t = std::chrono::steady_clock::now();
    char b[48];
    std::snprintf(b, sizeof(b), "%s%s=%.1f", phases.empty() ? "" : " ", name,
                  std::chrono::duration<double, std::milli>(t - tp).count());
    phases += b;
    tp = t;
  };
  try {
    std::call_once(placed_, [this] { place_on_gpu(); });
    if (gpu::device_count() <= 0) return;
    const int device = device_;
    if (hipSetDevice(device) != hipSuccess) return;
    lap("hip");
    try {
      (void)gpu::SdmaEngine::for_device(device);
    } catch (const std::exception&) {
    }
    lap("sdma");
    warm_code(device);
    lap("code");
    // a workspace with its pinned D2H ring (NUMA-local), and an early stager, into the device pools
    warm_workspaces(device, 1);
    if (pc.early_h2d) {
      PoolLease<EarlyStager> sl{device, DevicePool<EarlyStager>::get().acquire(
                                            device, [device] { return std::make_unique<EarlyStager>(device); })};
      sl.clean = true;
    }
    lap("ws");
    // TeraSort-shaped tasks merge through device_reduce_fixed: its pooled workspace, merger and SDMA
    // delivery ring
    {
      gpu::DeviceReduceConfig cfg;
      cfg.device = device;
      cfg.kv_buf_bytes = kv_buf_size_;
      cfg.round_bytes = pc.round_bytes;
      gpu::prewarm_device_reduce(cfg, std::max(1, pc.maps));
    }
    lap("fixed10");
    // pinned blocks for the fetch arena, kept in the pool's cache for this task's partitions (not for
    // tasks that only fetch device descriptors)
    const int64_t pin = pc.pinned_bytes;
    std::vector<gpu::PinnedPool::Block> blocks;
    for (int64_t b = 0; b < pin && !stop_; b += (int64_t)gpu::PinnedArena::kBlock)
      blocks.push_back(gpu::PinnedPool::instance().acquire(gpu::PinnedArena::kBlock));
    for (auto& b : blocks) gpu::PinnedPool::instance().release(b);
    lap("pinned");
  } catch (const std::exception& e) {
    UDA_LOG(kWarn, "GPU prewarm: %s", e.what());
  }
  std::lock_guard<std::mutex> g(st_mu_);
  st_.gpu_prewarm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  st_.gpu_prewarm_phases = phases;
}

void ReduceTask::join_prewarm() {
  // placed by the prewarm; without one (or if it failed there) here, where a failure fails the task
  if (!prewarm_thr_.joinable()) {
    std::call_once(placed_, [this] { place_on_gpu(); });
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  prewarm_thr_.join();
  std::call_once(placed_, [this] { place_on_gpu(); });
  std::lock_guard<std::mutex> g(st_mu_);
  st_.gpu_prewarm_wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void ReduceTask::merge_gpu() {
  join_prewarm();
  if (gpu::device_count() <= 0) throw UdaError("mapred.uda.merge.backend=gpu but no HIP device is visible");
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.merge_path = "staged";
  }
  auto t0 = std::chrono::steady_clock::now();
  const int maps = init_.num_maps;
  const int device = device_;
  if (hipSetDevice(device) != hipSuccess) throw UdaError("hipSetDevice failed");
  GateLease gate;
  // Off by default: a gated task fetches nothing until all its FETCHes are in, which under reduce
  // slow-start gives up the fetch / map-phase overlap. With every map output already there, 16
  // concurrent host-MOF TeraSort tasks reach 20.8 GB/s unlimited and 31.2 / 34.3 / 32.6 with 4 / 6 / 8
  // slots (profiles/r2_api_host_mofs_gate_sweep.md): set it for jobs whose reduces start after the maps.
  if (const int cap = (int)host_->conf_i64("mapred.uda.gpu.max.concurrent.merges", 0); cap > 0) {
    const auto w0 = std::chrono::steady_clock::now();
    // A task asks for a slot only once every map has been announced (all FETCH commands in): a task
    // still waiting for map outputs (reduce slow-start) must not hold a slot, and a host that feeds the
    // tasks' FETCHes one task after another cannot deadlock against the gate.
    {
      std::unique_lock<std::mutex> lk(mu_);
      while (!stop_ && !final_ && fetch_cmds_ < maps) cv_.wait_for(lk, std::chrono::milliseconds(50));
    }
    if (!DeviceGate::get().acquire(device, cap, [&] { return stop_.load(); }))
      throw UdaError("reduce task stopped while waiting for a GPU merge slot");
    gate.device = device;
    std::lock_guard<std::mutex> g(st_mu_);
    st_.gpu_gate_wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  }
  const bool device_decode = codec_ != Codec::kNone && host_->conf_i64("mapred.uda.gpu.decompress", 1) != 0;
  const Codec fetch_codec = device_decode ? Codec::kNone : codec_;
  const Codec stage_codec = device_decode ? codec_ : Codec::kNone;
  // device budget per merge: in + out + elements + side tables ~ 3x the input
  int64_t budget = host_->conf_i64("mapred.uda.gpu.merge.bytes", 0);
  if (budget <= 0) {
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    budget = (int64_t)(free_b / 4);
  }
  // and within the device's HBM budget (mapred.uda.gpu.hbm.budget, hbm_ledger.h): three pipelined RPQ
  // rounds of budget/2 input, each workspace ~3x its input, come to ~4.5x the input budget (the stager's
  // blocks are released at the switch to direct rounds)
  {
    const int64_t hr = gpu::HbmLedger::get().headroom(device);
    if (hr > 0 && budget > hr / 5) {
      budget = std::max<int64_t>(hr / 5, 64ll << 20);
      std::lock_guard<std::mutex> g(st_mu_);
      st_.merge_budget_from_ledger = 1;
    }
  }
  const std::string tier = host_->get_conf("mapred.uda.gpu.spill", init_.local_dirs.empty() ? "host" : "disk");
  StreamGuard sg;
  sg.s = gpu::pooled_stream();
  hipStream_t s = sg.s;
  PoolLease<DeviceWorkspace> ws_lease{device, DevicePool<DeviceWorkspace>::get().acquire(
                                                  device, [] { return std::make_unique<DeviceWorkspace>(); })};
  DeviceWorkspace& ws = *ws_lease.obj;
  ws.reset_stats();
  PoolLease<DeviceWorkspace> ws2_lease{device, nullptr}, ws3_lease{device, nullptr};  // pipelined RPQ rounds
  DeviceWorkspace* ws2 = nullptr;
  DeviceWorkspace* ws3 = nullptr;
  // uncompressed partitions go to HBM as soon as each one is complete (overlapping the fetch)
  // Two stagers: the group being fetched is staged by `stager` while the LPQ thread merges the
  // previous group out of `job_stager`'s arena; spill_group swaps them.
  PoolLease<EarlyStager> stager_lease{device, nullptr}, stager_lease2{device, nullptr};
  EarlyStager* stager = nullptr;
  EarlyStager* job_stager = nullptr;
  if (fetch_codec == Codec::kNone && stage_codec == Codec::kNone && host_->conf_i64("mapred.uda.gpu.early.h2d", 1) != 0) {
    stager_lease.obj = DevicePool<EarlyStager>::get().acquire(device, [device] { return std::make_unique<EarlyStager>(device); });
    stager = stager_lease.obj.get();
    stager->reset();
  }
  const int depth = (int)std::max<int64_t>(1, host_->conf_i64("mapred.uda.gpu.fetch.depth", 4));
  // early staging granularity: <= 0 (default) copies each partition once it is complete; > 0 copies
  // every `step` bytes of its landed prefix. Measured on the 2 GB secondary sort, 8 MiB pieces made the
  // fetch 70-200 ms instead of 21-25 ms (either copy path, SDMA or blit), while a standalone probe
  // (tools/host_dma_contention.py) shows CPU copies into pinned memory unaffected by a concurrent H2D;
  // the cause is not understood, so piecewise staging stays opt-in.
  const int64_t stage_step = host_->conf_i64("mapred.uda.gpu.early.h2d.step", 0);
  // MOFs drained at once (0: all that have arrived). 8 keeps partitions completing one after another,
  // so each one's H2D overlaps the remaining fetch: 2 GB secondary sort 23.3 GB/s vs 12.7-21 with all 64.
  const int64_t drains = host_->conf_i64("mapred.uda.gpu.fetch.drains", 8);

  std::vector<SpillRun> spills;
  std::vector<Span> group;          // fetched partitions of the current group (pinned, group_mem)
  gpu::PinnedArena group_mem, spill_mem;
  int64_t group_raw = 0;
  std::unique_ptr<AsyncIO> aio;
  std::vector<std::string> dirs = init_.local_dirs;
  if (dirs.empty()) dirs.push_back("/tmp");
  // LPQ checkpoint (disk tier): spills[0, checkpointed) are fsynced, indexed in <path>.idx and
  // listed in the manifest; a failed attempt keeps them for the next one
  const bool ckpt = checkpoint_ && tier == "disk";
  // Progressive merge (mapred.uda.gpu.progressive.phases = P > 1, online tasks whose whole input fits
  // the device budget): every partition is fetched in P byte phases, all partitions' phase p before
  // any phase p + 1, each phase staged to HBM as it lands. After phase p the key range below the least
  // last-landed key has fully arrived in every run (plan_progressive_split), so it is merged and its
  // output streamed back while phase p + 1 still comes in: the D2H of the output overlaps the H2D of
  // the input on the duplex link instead of following it.
  // Default (-1): 4 phases when the task is the only staged GPU merge on its device when it decides
  // (a lone task: 22 -> 26.3-26.8 GB/s on the 2 GB secondary sort); concurrent tasks already overlap
  // each other's H2D and D2H and gain nothing (profiles/r3_api_host_mofs_progressive_ab.txt).
  const int64_t prog_conf = host_->conf_i64("mapred.uda.gpu.progressive.phases", -1);
  const int prog_phases = (int)std::min<int64_t>(EarlyStager::kGroups, prog_conf < 0 ? 4 : prog_conf);
  const bool prog_auto = prog_conf < 0;
  StagedCount staged_count(device);
  const bool prog_ok = prog_phases > 1 && stager && stager->sdma() && restored_files_.empty() && !ckpt;
  // over budget, DRAM tier: phases into pinned DRAM, RPQ rounds of every fully arrived key range (DirectProg)
  const int pdirect_phases = (int)std::max<int64_t>(1, host_->conf_i64("mapred.uda.gpu.hybrid.progressive.phases", 16));
  bool prog_decided = false, progressive = false;
  struct ProgFetch {
    int P = 0, K = 0;
    std::vector<std::shared_ptr<MofFetcher>> f;
    std::vector<uint8_t*> dst, dev;
    std::vector<int64_t> cap;
    std::vector<std::vector<int64_t>> landed;  // [phase][run]: end of the bytes that phase fetched
    std::vector<int> done;                     // per phase: partitions whose phase is fetched and queued to HBM
    std::mutex mu;
    std::condition_variable cv;
    std::exception_ptr err;
    std::atomic<int64_t> next{0};
    std::vector<std::thread> threads;
    std::chrono::steady_clock::time_point t_end;
    ~ProgFetch() {
      for (auto& t : threads)
        if (t.joinable()) t.join();
    }
  };
  std::unique_ptr<ProgFetch> prog;
  // Progressive direct RPQ (mapred.uda.gpu.hybrid.progressive, default on): a task whose input outgrows
  // the device budget on the DRAM tier fetches every partition in P byte phases into pinned DRAM, and the
  // fetch threads index each run as its phases land (in order per run). After phase p the key range below
  // the least last-complete key of the unfinished runs has fully arrived in every run: it is merged in
  // RPQ rounds (slices H2D, merge, D2H, as the direct RPQ) while later phases still come in. Without it
  // the RPQ rounds start after the last byte landed (the reference's fetcher-ahead-of-LPQ pipeline,
  // MergeManager.cc:202-288, is what this recovers).
  struct DirectProg {
    int P = 0, K = 0;
    int64_t spacing = kSampleSpacing;        // index sample spacing of the runs
    std::vector<std::shared_ptr<MofFetcher>> f;
    std::vector<uint8_t*> dst;
    std::vector<int64_t> cap;
    std::vector<std::vector<char>> fetched;  // [k][p]
    std::vector<int> indexed;                // [k]: phases of run k indexed
    std::vector<char> indexing;              // [k]: a thread is indexing run k
    std::vector<RunCursor> cur;              // [k]: touched by the thread indexing run k only
    std::vector<std::vector<int64_t>> cut;   // [k]: samples so far (appended under mu)
    std::vector<std::vector<std::string>> key;
    std::vector<int64_t> complete;           // [k]: end of the last complete record indexed
    std::vector<std::string> last_key;       // [k]: key of that record ("" none yet)
    std::vector<char> eof;                   // [k]: the partition is indexed to its EOF marker
    std::vector<int> phase_runs;             // [p]: runs indexed through phase p
    std::vector<gpu::PinnedPool::Block> blocks;  // [k]: the pinned span of partition k (back to the pool at the end)
    std::mutex mu;
    std::condition_variable cv;
    std::exception_ptr err;
    std::atomic<int64_t> next{0};
    std::vector<std::thread> threads;
    std::chrono::steady_clock::time_point t_end;
    ~DirectProg() {
      for (auto& t : threads)
        if (t.joinable()) t.join();
      for (auto& b : blocks) gpu::PinnedPool::instance().release(b);
    }
  };
  std::unique_ptr<DirectProg> dprog;
  const std::string manifest = ckpt ? checkpoint_path() : std::string();
  size_t checkpointed = 0;
  std::vector<std::string> group_ids;  // MOFs of the current group (for the manifest)
  auto cleanup = [&](bool ok) {
    for (size_t i = 0; i < spills.size(); ++i) {
      SpillRun& r = spills[i];
      if (r.fd >= 0) ::close(r.fd);
      const bool keep = !ok && ckpt && i < checkpointed;
      if (!r.path.empty() && !keep) {
        ::unlink(r.path.c_str());
        if (ckpt) ::unlink((r.path + ".idx").c_str());
      }
      r.fd = -1;
      r.path.clear();
    }
    if (ok && ckpt) ::unlink(manifest.c_str());
  };
  auto count_decoded = [&](int64_t n) {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.device_decoded_blocks += n;
  };
  // LPQ: merge the current group on the device and spill it with its sparse index
  // LPQ: merge one group on the device and spill it with its sparse index. Runs on the LPQ thread,
  // one group at a time, while the fetch fills the next group (the reference's fetcher running ahead
  // of the LPQ merges, MergeManager.cc:202-288).
  auto merge_spill = [&](std::vector<Span> jg, std::vector<std::string> ids, EarlyStager* st) {
    const int64_t tl = trace::host_enabled() ? trace::now_ns() : 0;
    if (st) st->flush();
    const int64_t tm = tl ? trace::now_ns() : 0;
    DeviceMergeOut m = device_merge(ws, jg, stage_codec, kind_, kSampleSpacing, s);
    if (tl) {
      trace::host_event("lpq_flush", (int64_t)jg.size(), 0, tl, tm);
      trace::host_event("lpq_merge", m.bytes, (int64_t)jg.size(), tm, trace::now_ns());
    }
    count_decoded(m.decoded_blocks);
    if (st) st->reset();  // the merge read the staged copies; recycle their HBM
    SpillRun run;
    run.bytes = m.bytes;
    const bool disk = tier == "disk";
    if (disk) {
      if (!aio) aio = AsyncIO::create(AsyncIO::Options{});
      char name[64];
      snprintf(name, sizeof(name), ".gpu-lpq-%03d", (int)spills.size());
      run.path = dirs[spills.size() % dirs.size()] + "/uda." + init_.reduce_task_id + name;
      run.fd = create_private_file(run.path, O_RDWR);
      if (run.fd < 0) throw UdaError("cannot create spill file " + run.path + ": " + strerror(errno));
    } else {
      run.mem = spill_mem.alloc((size_t)std::max<int64_t>(run.bytes, 1));
    }
    // stream the LPQ output out of HBM: sparse index from every cut, bytes to DRAM or to the file.
    // The DRAM tier is pinned, so the LPQ lands there by one DMA (no bounce through the ring).
    std::atomic<int64_t> err{0};
    if (!disk) {
      const auto td = std::chrono::steady_clock::now();
      const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
      // on the SDMA delivery engine (idle until the RPQ rounds deliver), not a blit kernel on the CUs
      // the next LPQ merge needs; device_merge returned with `s` drained
      gpu::SdmaEngine* eng = nullptr;
      if (m.bytes > 0) {
        try {
          eng = &gpu::SdmaEngine::for_device(device);
        } catch (const std::exception&) {
          eng = nullptr;
        }
      }
      if (eng) {
        if (!ws.h2d_sig.handle) ws.h2d_sig = eng->make_signal();
        gpu::SdmaEngine::arm(ws.h2d_sig, eng->parts((size_t)m.bytes, 1));
        eng->copy_d2h(run.mem, ws.out.as<uint8_t>(), (size_t)m.bytes, ws.h2d_sig, 1);
        gpu::SdmaEngine::wait(ws.h2d_sig);
      } else if (m.bytes > 0) {
        HIP_CHECK(hipMemcpyAsync(run.mem, ws.out.as<uint8_t>(), (size_t)m.bytes, hipMemcpyDeviceToHost, s));
      }
      HIP_CHECK(hipStreamSynchronize(s));
      if (tt) trace::host_event("lpq_d2h", m.bytes, 0, tt, trace::now_ns());
      ws.d2h_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count();
      for (size_t j = 0; j + 1 < m.cuts.size(); ++j) {
        run.cut.push_back(m.cuts[j]);
        run.key.push_back(key_at(run.mem + m.cuts[j], m.cuts[j + 1] - m.cuts[j]));
      }
    } else
    stream_out(ws, m, s, [&](const uint8_t* p, size_t c0, size_t c1) {
      const int64_t base = m.cuts[c0], len = m.cuts[c1] - base;
      for (size_t j = c0; j < c1; ++j) {
        run.cut.push_back(m.cuts[j]);
        run.key.push_back(key_at(p + (m.cuts[j] - base), m.cuts[c1] - m.cuts[j]));
      }
      if (disk) {
        constexpr int64_t kIo = 8 << 20;
        for (int64_t o = 0; o < len; o += kIo)
          aio->write(run.fd, base + o, std::min(kIo, len - o), p + o, [&err](int64_t r) {
            if (r < 0) err = r;
          });
        aio->drain();  // the pinned piece is reused after this returns
      } else {
        std::memcpy(run.mem + base, p, (size_t)len);
      }
    });
    if (err.load() < 0) throw UdaError("spill write failed: " + std::string(strerror((int)-err.load())));
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.lpqs++;
      st_.spill_bytes += run.bytes;
    }
    const std::string run_path = run.path;
    const int run_fd = run.fd;
    std::vector<int64_t> idx_cut = ckpt ? run.cut : std::vector<int64_t>();
    std::vector<std::string> idx_key = ckpt ? run.key : std::vector<std::string>();
    const int64_t run_bytes = run.bytes;
    spills.push_back(std::move(run));
    if (ckpt && disk) {
      // durable before listed: data, then the sparse index, then the manifest line
      if (::fsync(run_fd) != 0) throw UdaError("spill fsync failed");
      const std::string ip = run_path + ".idx";
      {
        std::string ix;
        const int64_t n = (int64_t)idx_cut.size();
        ix.append(reinterpret_cast<const char*>(&n), 8);
        for (size_t j = 0; j < idx_cut.size(); ++j) {
          const int32_t kl = (int32_t)idx_key[j].size();
          ix.append(reinterpret_cast<const char*>(&idx_cut[j]), 8);
          ix.append(reinterpret_cast<const char*>(&kl), 4);
          ix.append(idx_key[j].data(), (size_t)kl);
        }
        const int ifd = create_private_file(ip, O_WRONLY);
        const bool ok = ifd >= 0 && write_all(ifd, ix.data(), ix.size()) && ::fsync(ifd) == 0;
        if (ifd >= 0) ::close(ifd);
        if (!ok) throw UdaError("cannot write LPQ index " + ip);
      }
      std::string line = "glpq " + std::to_string(spills.size() - 1) + " " + std::to_string(run_bytes) + " " + run_path + " ";
      for (size_t j = 0; j < ids.size(); ++j) line += (j ? "," : "") + ids[j];
      if (!append_owned_line(manifest, line)) throw UdaError("cannot append to LPQ manifest " + manifest);
      checkpointed = spills.size();
      if (fault_hit("LPQ_DONE")) throw UdaError("injected failure after an LPQ spill");
    }
  };
  // The group being fetched lives in fill_mem (and is staged to HBM by `stager`); the one being merged
  // in job_mem (its HBM copies in job_stager's arena), so the next group's H2D overlaps an LPQ merge.
  gpu::PinnedArena group_mem2;
  gpu::PinnedArena* fill_mem = &group_mem;
  gpu::PinnedArena* job_mem = &group_mem2;
  std::thread lpq_thr;
  std::exception_ptr lpq_err;
  auto lpq_wait = [&] {
    if (lpq_thr.joinable()) lpq_thr.join();
    if (lpq_err) {
      std::exception_ptr e = lpq_err;
      lpq_err = nullptr;
      std::rethrow_exception(e);
    }
  };
  struct LpqJoin {
    std::thread& t;
    ~LpqJoin() {
      if (t.joinable()) t.join();
    }
  } lpq_join{lpq_thr};
  auto spill_group = [&] {
    if (group.empty()) return;
    lpq_wait();               // one LPQ merge at a time (device workspace, stream s)
    job_mem->release_all();   // the previous LPQ's inputs are merged
    std::swap(fill_mem, job_mem);
    if (stager && !job_stager) {  // first LPQ: the second stager (online merges never need one)
      stager_lease2.obj = DevicePool<EarlyStager>::get().acquire(device, [device] { return std::make_unique<EarlyStager>(device); });
      job_stager = stager_lease2.obj.get();
      job_stager->reset();
    }
    std::swap(stager, job_stager);  // the group's staged copies go with it; the next group stages into the other
    std::vector<Span> jg;
    jg.swap(group);
    std::vector<std::string> ids;
    ids.swap(group_ids);
    group_raw = 0;
    EarlyStager* st = job_stager;
    lpq_thr = std::thread([&, device, st, jg = std::move(jg), ids = std::move(ids)]() mutable {
      try {
        if (hipSetDevice(device) != hipSuccess) throw UdaError("hipSetDevice failed");
        merge_spill(std::move(jg), std::move(ids), st);
      } catch (...) {
        lpq_err = std::current_exception();
      }
    });
  };
  // Direct RPQ (mapred.uda.gpu.hybrid.direct, default on, DRAM tier, uncompressed partitions, at most
  // mapred.uda.gpu.hybrid.direct.max.runs maps): once the input outgrows the device budget, the
  // fetched partitions stay where the fetch put them (pinned DRAM, already sorted runs) and are indexed
  // by the drain threads; the RPQ key-range rounds then merge slices of all of them. The reference's
  // LPQ level (MergeManager.cc:202-288) bounds a CPU heap's fan-in and spills to disk; on this tier it
  // would only re-sort bytes already in DRAM, at two extra PCIe crossings (LPQ H2D + spill D2H), while
  // the device K-way merge takes hundreds of runs per round. The disk tier keeps the LPQ level.
  const bool direct_ok = tier == "host" && codec_ == Codec::kNone && restored_files_.empty() && !ckpt &&
                         host_->conf_i64("mapred.uda.gpu.hybrid.direct", 1) != 0 &&
                         maps <= host_->conf_i64("mapred.uda.gpu.hybrid.direct.max.runs", 1024);
  const bool pdirect_ok = direct_ok && pdirect_phases > 1 && host_->conf_i64("mapred.uda.gpu.hybrid.progressive", 1) != 0;
  bool direct = false;
  std::vector<SpillRun> direct_runs;  // one per partition drained after the switch, in `group` order
  auto index_spans = [&](const std::vector<Span>& spans, size_t first, std::vector<SpillRun>* out) {
    const size_t n = spans.size() - first;
    out->resize(n);
    std::atomic<size_t> nk{0};
    std::vector<std::exception_ptr> errs(n);
    std::vector<std::thread> ts;
    // half the drain threads: this runs beside them (and the provider's) under the task's CPU share
    const size_t nt = std::min<size_t>(n, (size_t)std::max<int64_t>(1, (drains > 0 ? drains : 8) / 2));
    for (size_t w = 0; w < nt; ++w)
      ts.emplace_back([&] {
        for (size_t k; (k = nk++) < n;) try {
            (*out)[k] = index_host_run(const_cast<uint8_t*>(spans[first + k].p), spans[first + k].len, kSampleSpacing);
          } catch (...) {
            errs[k] = std::current_exception();
          }
      });
    for (auto& t : ts) t.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  };
  std::future<std::vector<SpillRun>> direct_head;  // partitions drained before the switch, indexed meanwhile
  // The group overflowed the budget: an LPQ merge, or the switch to direct RPQ (partitions drained so
  // far are indexed here, later ones by their drain threads; early staging to HBM stops).
  auto overflow = [&] {
    if (!direct_ok) {
      spill_group();
      return;
    }
    if (direct) return;
    direct = true;
    if (stager) {
      stager->release_blocks();  // the partitions' HBM copies are not used: RPQ rounds copy their slices
      stager = nullptr;
    }
    // indexed beside the fetch (which goes on filling `group`; the spans indexed here are a copy)
    direct_head = std::async(std::launch::async, [&index_spans, head = group] {
      std::vector<SpillRun> idx;
      index_spans(head, 0, &idx);
      return idx;
    });
    std::lock_guard<std::mutex> g(st_mu_);
    st_.hybrid_direct = 1;
  };
  // resume: restored LPQ spills (data + sparse index) of a failed attempt
  if (ckpt && restored_files_.empty()) ::unlink(manifest.c_str());
  for (const std::string& path : restored_files_) {
    SpillRun run;
    run.path = path;
    run.fd = ::open(path.c_str(), O_RDWR | O_CLOEXEC);
    struct stat sb;
    if (run.fd < 0 || ::fstat(run.fd, &sb) != 0) throw UdaError("cannot reopen checkpointed LPQ " + path);
    run.bytes = (int64_t)sb.st_size;
    std::ifstream ix(path + ".idx", std::ios::binary);
    int64_t n = -1;
    ix.read(reinterpret_cast<char*>(&n), 8);
    if (!ix || n < 0) throw UdaError("bad LPQ index " + path + ".idx");
    for (int64_t j = 0; j < n; ++j) {
      int64_t c = 0;
      int32_t kl = 0;
      ix.read(reinterpret_cast<char*>(&c), 8);
      ix.read(reinterpret_cast<char*>(&kl), 4);
      if (!ix || kl < 0) throw UdaError("bad LPQ index " + path + ".idx");
      std::string k((size_t)kl, '\0');
      ix.read(&k[0], kl);
      run.cut.push_back(c);
      run.key.push_back(std::move(k));
    }
    spills.push_back(std::move(run));
  }
  checkpointed = spills.size();
  if (!spills.empty()) {
    if (!aio) aio = AsyncIO::create(AsyncIO::Options{});
    std::lock_guard<std::mutex> g(st_mu_);
    st_.restored_lpqs = (int64_t)spills.size();
    st_.restored_maps = (int64_t)restored_maps_.size();
    st_.maps_fetched += (int64_t)restored_maps_.size();
  }

  try {
    // ---- fetch: start every MOF (bounded by the buffer pool), drain each fully into host memory
    std::mt19937_64 rng((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count());
    int started = (int)restored_maps_.size(), drained = started;
    total_count_ += started;
    if (started > 0 && total_count_ == maps) host_->fetch_over();
    std::vector<FetchParams> pending;
    std::vector<std::shared_ptr<MofFetcher>> ready;
    while (drained < maps) {
      std::vector<std::shared_ptr<MofFetcher>> to_start;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          return stop_ || !fetched_.empty() ||
                 ((!fetch_list_.empty() || !pending.empty()) && free_pairs_ > 0 && started < maps);
        });
        if (stop_) throw UdaError("reduce task stopped during fetch");
        while (!fetch_list_.empty()) {
          pending.push_back(fetch_list_.front());
          fetch_list_.pop_front();
        }
        std::shuffle(pending.begin(), pending.end(), rng);
        while (!pending.empty() && free_pairs_ > 0 && started < maps) {
          to_start.push_back(std::make_shared<MofFetcher>(this, pending.back(), buffer_size_, fetch_codec));
          pending.pop_back();
          free_pairs_--;
          started++;
        }
        while (!fetched_.empty()) {
          ready.push_back(fetched_.front());
          fetched_.pop_front();
        }
      }
      for (auto& f : to_start) f->start();
      if ((prog_ok || pdirect_ok) && !prog_decided) {
        if (drained + (int)ready.size() < maps) continue;  // every partition's length before deciding
        prog_decided = true;
        int64_t tot = 0;
        for (auto& f : ready) tot += std::max<int64_t>(f->part_len(), 0);
        progressive = prog_ok && drained == 0 && tot <= budget && (!prog_auto || staged_merges(device).load() == 1);
        if (!progressive && pdirect_ok && drained == 0 && tot > budget) {
          {
            std::lock_guard<std::mutex> g(st_mu_);
            st_.merge_path = "staged-progressive-direct";
            st_.hybrid_direct = 1;
          }
          if (stager) {  // the partitions never go to HBM whole: RPQ rounds copy their slices
            stager->release_blocks();
            stager = nullptr;
          }
          // the partitions' pinned spans come back to the pool when the task ends: keep them cached for the
          // next task of this size instead of re-pinning them
          gpu::PinnedPool::instance().raise_cache_cap((size_t)(tot + tot / 8));
          dprog = std::make_unique<DirectProg>();
          DirectProg& dp = *dprog;
          dp.P = pdirect_phases;
          dp.K = (int)ready.size();
          // samples fine enough that a round of budget/2 can be cut from K runs (a few per run and round):
          // 256 KiB for GB partitions, finer for small tasks under a small budget
          dp.spacing = std::clamp<int64_t>(budget / 2 / (4 * std::max(1, dp.K)), 4 << 10, kSampleSpacing);
          dp.f = ready;
          for (auto& f : ready) dp.cap.push_back(std::max<int64_t>(f->part_len(), 0));
          const size_t K = (size_t)dp.K;
          // each partition's pinned span is taken by the thread that fetches its first phase (in parallel,
          // beside the first fetches: pinning GBs serially here held up the whole fetch)
          dp.dst.assign(K, nullptr);
          dp.blocks.assign(K, gpu::PinnedPool::Block{});
          dp.fetched.assign(K, std::vector<char>((size_t)dp.P, 0));
          dp.indexed.assign(K, 0);
          dp.indexing.assign(K, 0);
          dp.cur.assign(K, RunCursor());
          dp.cut.assign(K, {});
          dp.key.assign(K, {});
          dp.complete.assign(K, 0);
          dp.last_key.assign(K, std::string());
          dp.eof.assign(K, 0);
          dp.phase_runs.assign((size_t)dp.P, 0);
          auto work = [this, &dp, depth] {
            for (int64_t i; (i = dp.next++) < (int64_t)dp.P * dp.K;) {
              {
                std::lock_guard<std::mutex> g(dp.mu);
                if (stop_ || dp.err) break;
              }
              const int p = (int)(i / dp.K), k = (int)(i % dp.K);
              try {
                MofFetcher& f = *dp.f[(size_t)k];
                const int64_t cap = dp.cap[(size_t)k];
                const int64_t b = cap * p / dp.P, e = cap * (p + 1) / dp.P;
                if (p == 0) {
                  const gpu::PinnedPool::Block blk = gpu::PinnedPool::instance().acquire((size_t)std::max<int64_t>(cap, 256));
                  {
                    std::lock_guard<std::mutex> g(dp.mu);
                    dp.blocks[(size_t)k] = blk;
                    dp.dst[(size_t)k] = blk.p;
                    dp.cv.notify_all();
                  }
                  const int64_t off = f.take_first(dp.dst[(size_t)k], cap);
                  if (off < e) fetch_direct(f.params(), dp.dst[(size_t)k], off, e, depth, nullptr, 0);
                } else if (b < e) {
                  {  // its first phase (another thread) may still be taking the span
                    std::unique_lock<std::mutex> lk(dp.mu);
                    dp.cv.wait(lk, [&] { return dp.dst[(size_t)k] != nullptr || dp.err; });
                    if (dp.err) break;
                  }
                  fetch_direct(f.params(), dp.dst[(size_t)k], b, e, depth, nullptr, 0);
                }
                // index run k through every phase landed in order (one thread per run at a time)
                std::unique_lock<std::mutex> lk(dp.mu);
                dp.fetched[(size_t)k][(size_t)p] = 1;
                while (!dp.indexing[(size_t)k] && dp.indexed[(size_t)k] < dp.P &&
                       dp.fetched[(size_t)k][(size_t)dp.indexed[(size_t)k]]) {
                  dp.indexing[(size_t)k] = 1;
                  const int q = dp.indexed[(size_t)k];
                  const int64_t limit = cap * (q + 1) / dp.P;
                  lk.unlock();
                  std::vector<int64_t> c;
                  std::vector<std::string> kk;
                  RunCursor& rc = dp.cur[(size_t)k];
                  rc.advance(dp.dst[(size_t)k], limit, dp.spacing, &c, &kk);
                  std::string lkey = rc.last_key(dp.dst[(size_t)k]);
                  lk.lock();
                  auto& vc = dp.cut[(size_t)k];
                  auto& vk = dp.key[(size_t)k];
                  vc.insert(vc.end(), c.begin(), c.end());
                  for (auto& x : kk) vk.push_back(std::move(x));
                  dp.complete[(size_t)k] = rc.pos;
                  if (!lkey.empty()) dp.last_key[(size_t)k] = std::move(lkey);
                  if (rc.eof || q + 1 == dp.P) dp.eof[(size_t)k] = 1;
                  dp.indexed[(size_t)k] = q + 1;
                  dp.indexing[(size_t)k] = 0;
                  if (++dp.phase_runs[(size_t)q] == dp.K && q + 1 == dp.P) dp.t_end = std::chrono::steady_clock::now();
                  dp.cv.notify_all();
                }
              } catch (...) {
                std::lock_guard<std::mutex> g(dp.mu);
                if (!dp.err) dp.err = std::current_exception();
                dp.cv.notify_all();
              }
            }
          };
          // fetch threads: enough to stay ahead of the merge, few enough not to slow the consumer they overlap
          const int64_t pt = host_->conf_i64("mapred.uda.gpu.hybrid.progressive.threads", drains > 0 ? drains : 8);
          const int nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(pt, dp.K));
          for (int w = 0; w < nthreads; ++w) dp.threads.emplace_back(work);
          drained = maps;
          ready.clear();
          continue;
        }
        if (progressive) {
          {
            std::lock_guard<std::mutex> g(st_mu_);
            st_.merge_path = "staged-progressive";
          }
          prog = std::make_unique<ProgFetch>();
          ProgFetch& pf = *prog;
          pf.P = prog_phases;
          pf.K = (int)ready.size();
          pf.f = ready;
          for (auto& f : ready) {
            const int64_t cap = std::max<int64_t>(f->part_len(), 0);
            pf.cap.push_back(cap);
            pf.dst.push_back(fill_mem->alloc((size_t)std::max<int64_t>(cap, 1)));
            pf.dev.push_back(stager->reserve(cap));
          }
          pf.landed.assign((size_t)pf.P, std::vector<int64_t>((size_t)pf.K, 0));
          pf.done.assign((size_t)pf.P, 0);
          EarlyStager* st = stager;
          auto work = [this, &pf, st, depth] {
            for (int64_t i; (i = pf.next++) < (int64_t)pf.P * pf.K;) {
              {
                std::lock_guard<std::mutex> g(pf.mu);
                if (stop_ || pf.err) break;  // a stopped or failed task fetches no further phases
              }
              const int p = (int)(i / pf.K), k = (int)(i % pf.K);
              int64_t e = 0;
              try {
                MofFetcher& f = *pf.f[(size_t)k];
                const int64_t cap = pf.cap[(size_t)k];
                const int64_t b = cap * p / pf.P;
                e = cap * (p + 1) / pf.P;
                if (p == 0) {
                  const int64_t off = f.take_first(pf.dst[(size_t)k], cap);
                  if (off < e) fetch_direct(f.params(), pf.dst[(size_t)k], off, e, depth, nullptr, 0);
                  e = std::max(e, off);
                  st->copy(pf.dst[(size_t)k], pf.dev[(size_t)k], e, 0);
                } else if (b < e) {  // (may refetch bytes the first chunk already brought: same bytes)
                  fetch_direct(f.params(), pf.dst[(size_t)k], b, e, depth, nullptr, 0);
                  st->copy(pf.dst[(size_t)k] + b, pf.dev[(size_t)k] + b, e - b, p);
                }
              } catch (...) {
                std::lock_guard<std::mutex> g(pf.mu);
                if (!pf.err) pf.err = std::current_exception();
              }
              std::lock_guard<std::mutex> g(pf.mu);
              pf.landed[(size_t)p][(size_t)k] = e;
              if (++pf.done[(size_t)p] == pf.K && p + 1 == pf.P) pf.t_end = std::chrono::steady_clock::now();
              pf.cv.notify_all();
            }
          };
          const int nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(drains > 0 ? drains : 8, pf.K));
          for (int w = 0; w < nthreads; ++w) pf.threads.emplace_back(work);
          drained = maps;  // the phases run on pf.threads; the merge below consumes them
          ready.clear();
          continue;
        }
      }
      // Drain arrived MOFs in parallel (each drain keeps one request in flight ahead) straight into
      // pinned spans of the group arena. Group boundaries are decided before a MOF is drained (on
      // its partition length), so a group is complete in host memory when it is merged and spilled.
      size_t next = 0;
      while (next < ready.size()) {
        std::vector<size_t> sub;
        while (next < ready.size()) {
          const int64_t pl = std::max<int64_t>(ready[next]->part_len(), 0);
          const int64_t est = pl * (codec_ != Codec::kNone ? 3 : 1);  // decoded size estimate
          if (!direct && (!group.empty() || !sub.empty()) && group_raw + est > budget) break;
          sub.push_back(next++);
          group_raw += est;
        }
        if (sub.empty()) {  // the group is full: merge and spill it (or go direct), then admit the MOF
          overflow();
          continue;
        }
        const bool index_now = direct;  // direct RPQ: each drain thread indexes its partition
        std::vector<SpillRun> sub_idx(index_now ? sub.size() : 0);
        std::vector<Span> got(sub.size());
        std::vector<std::vector<uint8_t>> host_decoded(sub.size());
        std::vector<uint8_t*> dst(sub.size(), nullptr);
        std::vector<std::exception_ptr> errs(sub.size());
        for (size_t k = 0; k < sub.size(); ++k)
          if (fetch_codec == Codec::kNone)
            dst[k] = fill_mem->alloc((size_t)std::max<int64_t>(ready[sub[k]]->part_len(), 1));
        // drains > 0: that many drain threads take the MOFs in turn, so partitions complete one after
        // another and their H2D overlaps the rest of the fetch (all at once, they complete together)
        std::atomic<size_t> next_k{0};
        auto drain = [&](size_t k) {
            const int64_t td = trace::host_enabled() ? trace::now_ns() : 0;
            try {
              MofFetcher& f = *ready[sub[k]];
              if (dst[k]) {
                // first chunk from the fetcher, the rest straight into the pinned span
                // With early staging the partition is copied to HBM once complete, or (stage_step > 0)
                // every stage_step bytes of its landed prefix while the rest is still in flight.
                const int64_t cap = f.part_len();
                uint8_t* dev = stager ? stager->reserve(cap) : nullptr;
                int64_t off = f.take_first(dst[k], cap);
                if (dev && stage_step > 0) stager->copy(dst[k], dev, off);
                if (off < cap) {
                  std::function<void(int64_t, int64_t)> on_prefix;
                  if (dev && stage_step > 0)
                    on_prefix = [&, k, dev](int64_t a, int64_t b) { stager->copy(dst[k] + a, dev + a, b - a); };
                  off = fetch_direct(f.params(), dst[k], off, cap, depth, on_prefix, stage_step);
                }
                if (dev && stage_step <= 0) stager->copy(dst[k], dev, off);
                got[k] = Span{dst[k], off, dev};
                if (index_now) sub_idx[k] = index_host_run(dst[k], off, kSampleSpacing);
              } else {  // host decode: decoded length unknown up front
                std::vector<uint8_t> buf((size_t)buffer_size_);
                for (int64_t n; (n = f.pull(buf.data(), (int64_t)buf.size())) > 0;)
                  host_decoded[k].insert(host_decoded[k].end(), buf.begin(), buf.begin() + n);
              }
            } catch (...) {
              errs[k] = std::current_exception();
            }
            if (td) trace::host_event("drain", (int64_t)k, got[k].len, td, trace::now_ns());
        };
        std::vector<std::thread> ts;
        const size_t nthreads = drains > 0 ? std::min<size_t>((size_t)drains, sub.size()) : sub.size();
        for (size_t w = 0; w < nthreads; ++w)
          ts.emplace_back([&] {
            for (size_t k; (k = next_k++) < sub.size();) drain(k);
          });
        for (auto& t : ts) t.join();
        for (auto& e : errs)
          if (e) std::rethrow_exception(e);
        for (size_t k = 0; k < sub.size(); ++k) {
          if (!dst[k]) {
            uint8_t* p = fill_mem->alloc(std::max<size_t>(host_decoded[k].size(), 1));
            std::memcpy(p, host_decoded[k].data(), host_decoded[k].size());
            got[k] = Span{p, (int64_t)host_decoded[k].size()};
          }
          group.push_back(got[k]);
          if (index_now) direct_runs.push_back(std::move(sub_idx[k]));
          if (ckpt) group_ids.push_back(ready[sub[k]]->params().map_id);
          drained++;
          progress_count_++;
          total_count_++;
          {
            std::lock_guard<std::mutex> gl(st_mu_);
            st_.maps_fetched++;
          }
          if (progress_count_ == 20 || total_count_ == maps) {
            host_->fetch_over();
            progress_count_ = 0;
          }
        }
        if (next < ready.size()) overflow();  // the next MOF did not fit this group
      }
      ready.clear();
    }
    const double fetch_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stager && std::getenv("UDA_STAGE_TRACE"))
      std::fprintf(stderr, "[stage] fetch %.1f ms, early H2D (%s) %lld copies of %.1f MB issued in %.1f ms, step %lld\n",
                   fetch_ms, stager->engine(), (long long)stager->copies(), stager->bytes() / 1e6, stager->issue_ms(),
                   (long long)stage_step);

    if (trace::host_enabled()) trace::host_event("fetch_phase", stage_step, drains, trace::now_ns() - (int64_t)(fetch_ms * 1e6), trace::now_ns());
    // ---- delivery of merged rounds; EOF rides in the very last buffer
    bool eof_sent = false;
    std::vector<uint8_t> tail((size_t)kv_buf_size_ + kEofBytes);
    auto deliver = [&](const DeviceMergeOut& m, bool last, hipStream_t ds, DeviceWorkspace& w) {
      const size_t nb = m.cuts.size() < 2 ? 0 : m.cuts.size() - 1;
      stream_out(w, m, ds, [&](const uint8_t* piece, size_t c0, size_t c1) {
        for (size_t j = c0; j < c1; ++j) {
          if (stop_) throw UdaError("reduce task stopped during merge");
          const int64_t b = m.cuts[j], e = m.cuts[j + 1];
          const bool final_buf = last && j + 1 == nb;
          const uint8_t* p = piece + (b - m.cuts[c0]);
          int64_t len = e - b;
          if (final_buf) {  // copy so the EOF marker can follow the records
            std::memcpy(tail.data(), p, (size_t)len);
            tail[(size_t)len] = 0xFF;
            tail[(size_t)len + 1] = 0xFF;
            p = tail.data();
            len += kEofBytes;
            eof_sent = true;
          }
          if (host_->data_from_uda(p, (int32_t)len) != 0) throw UdaError("dataFromUda callback failed");
          std::lock_guard<std::mutex> g(st_mu_);
          st_.buffers++;
          st_.bytes_delivered += len;
        }
      });
      std::lock_guard<std::mutex> g(st_mu_);
      st_.records += m.records;
    };
    const int64_t kv = kv_buf_size_ - kEofBytes;

    lpq_wait();  // an LPQ of the fetch phase may still be merging
    double prog_fetch_ms = -1;
    if (dprog) {
      DirectProg& dp = *dprog;
      const int K = dp.K;
      // merge-owned views of the runs: the landed, indexed prefix of every partition
      std::vector<SpillRun> runs((size_t)K);  // .mem set once the fetch threads have pinned the spans
      std::vector<int64_t> at((size_t)K, 0);  // merged so far (a record boundary)
      std::vector<size_t> taken((size_t)K, 0);  // samples copied into runs[k]
      // first record of `run` (indexed prefix) whose key is >= k
      auto boundary = [&](const SpillRun& run, const std::string& k) -> int64_t {
        int lo = -1, hi = (int)run.cut.size();
        while (hi - lo > 1) {
          const int mid = (lo + hi) / 2;
          if (cmp_key(kind_, run.key[(size_t)mid], k) < 0)
            lo = mid;
          else
            hi = mid;
        }
        if (lo < 0) return 0;
        const int64_t b = run.cut[(size_t)lo];
        const int64_t e = (size_t)lo + 1 < run.cut.size() ? run.cut[(size_t)lo + 1] : run.bytes;
        int64_t p = 0;
        while (b + p < e) {
          RecordView rv;
          if (ifile_parse(run.mem + b + p, (size_t)(e - b - p), &rv) != Parse::kRecord)
            throw UdaError("progressive hybrid: bad record in an indexed prefix");
          if (key_compare(kind_, rv.key, rv.klen, reinterpret_cast<const uint8_t*>(k.data()), (int)k.size()) >= 0) break;
          p += rv.size();
        }
        return b + p;
      };
      // three workspaces, two rounds prepared ahead (as the direct RPQ below)
      ws2_lease.obj = DevicePool<DeviceWorkspace>::get().acquire(device, [] { return std::make_unique<DeviceWorkspace>(); });
      ws2 = ws2_lease.obj.get();
      ws2->reset_stats();
      ws3_lease.obj = DevicePool<DeviceWorkspace>::get().acquire(device, [] { return std::make_unique<DeviceWorkspace>(); });
      ws3 = ws3_lease.obj.get();
      ws3->reset_stats();
      StreamGuard sg2, sg3;
      sg2.s = gpu::pooled_stream();
      sg3.s = gpu::pooled_stream();
      DeviceWorkspace* wsv[3] = {&ws, ws2, ws3};
      hipStream_t sv[3] = {s, sg2.s, sg3.s};
      // every round is a list of per-run [b, e) slices of the pinned partitions; rounds queue up as the
      // phases land and the pipeline below takes them in order
      std::vector<std::vector<std::pair<int64_t, int64_t>>> rounds;
      bool planned_all = false;
      const int64_t target = std::max<int64_t>(budget / 2, dp.spacing);
      int epoch = 0;
      // plan the rounds of every key range that has fully arrived; false while nothing new can be planned
      auto plan_more = [&](bool wait) -> bool {
        std::unique_lock<std::mutex> lk(dp.mu);
        auto ready_epoch = [&] { return epoch < dp.P && dp.phase_runs[(size_t)epoch] == K; };
        if (wait)
          while (!dp.cv.wait_for(lk, std::chrono::milliseconds(50), [&] { return ready_epoch() || dp.err || stop_; })) {
          }
        if (dp.err) std::rethrow_exception(dp.err);
        if (stop_) throw UdaError("reduce task stopped during fetch");
        if (!ready_epoch()) return false;
        while (ready_epoch()) ++epoch;  // take every phase indexed by now
        bool all_eof = true, blocked = false;
        std::string bound;
        bool have_bound = false;
        for (int k = 0; k < K; ++k) {
          SpillRun& r = runs[(size_t)k];
          r.mem = dp.dst[(size_t)k];  // indexed through a phase: its span exists
          auto& vc = dp.cut[(size_t)k];
          auto& vk = dp.key[(size_t)k];
          for (size_t j = taken[(size_t)k]; j < vc.size(); ++j) {
            r.cut.push_back(vc[j]);
            r.key.push_back(vk[j]);
          }
          taken[(size_t)k] = vc.size();
          r.bytes = dp.complete[(size_t)k];
          if (dp.eof[(size_t)k]) continue;
          all_eof = false;
          if (dp.last_key[(size_t)k].empty()) {
            blocked = true;  // no complete record of this run yet: nothing below any bound is known
            continue;
          }
          if (!have_bound || cmp_key(kind_, dp.last_key[(size_t)k], bound) < 0) {
            bound = dp.last_key[(size_t)k];
            have_bound = true;
          }
        }
        lk.unlock();
        if (!all_eof && (blocked || !have_bound)) return true;  // wait for more phases
        std::vector<int64_t> end((size_t)K);
        for (int k = 0; k < K; ++k)
          end[(size_t)k] = all_eof ? runs[(size_t)k].bytes : std::max(at[(size_t)k], boundary(runs[(size_t)k], bound));
        // splitters every ~budget/2 bytes of the range (samples inside it, by key)
        struct Sample {
          int run;
          int idx;
        };
        std::vector<Sample> smp;
        for (int k = 0; k < K; ++k) {
          const SpillRun& r = runs[(size_t)k];
          for (int j = 0; j < (int)r.cut.size(); ++j)
            if (r.cut[(size_t)j] >= at[(size_t)k] && r.cut[(size_t)j] < end[(size_t)k]) smp.push_back({k, j});
        }
        std::stable_sort(smp.begin(), smp.end(), [&](const Sample& a, const Sample& b) {
          const int c = cmp_key(kind_, runs[(size_t)a.run].key[(size_t)a.idx], runs[(size_t)b.run].key[(size_t)b.idx]);
          return c != 0 ? c < 0 : (a.run != b.run ? a.run < b.run : a.idx < b.idx);
        });
        std::vector<std::string> split;
        int64_t acc = 0;
        for (const Sample& sm : smp) {
          const SpillRun& r = runs[(size_t)sm.run];
          const int64_t nx = std::min(end[(size_t)sm.run], (size_t)sm.idx + 1 < r.cut.size() ? r.cut[(size_t)sm.idx + 1] : r.bytes);
          if (acc >= target) {
            const std::string& kk = r.key[(size_t)sm.idx];
            if (split.empty() || cmp_key(kind_, split.back(), kk) < 0) {
              split.push_back(kk);
              acc = 0;
            }
          }
          acc += nx - r.cut[(size_t)sm.idx];
        }
        std::vector<std::vector<int64_t>> b((size_t)K);
        for (int k = 0; k < K; ++k) {
          b[(size_t)k].push_back(at[(size_t)k]);
          for (const auto& kk : split)
            b[(size_t)k].push_back(std::min(end[(size_t)k], std::max(b[(size_t)k].back(), boundary(runs[(size_t)k], kk))));
          b[(size_t)k].push_back(end[(size_t)k]);
        }
        for (size_t q = 0; q + 1 < b[0].size(); ++q) {
          std::vector<std::pair<int64_t, int64_t>> rr((size_t)K);
          int64_t bytes = 0;
          for (int k = 0; k < K; ++k) {
            rr[(size_t)k] = {b[(size_t)k][q], b[(size_t)k][q + 1]};
            bytes += rr[(size_t)k].second - rr[(size_t)k].first;
          }
          if (bytes > 0 || (all_eof && q + 2 == b[0].size())) rounds.push_back(std::move(rr));
        }
        for (int k = 0; k < K; ++k) at[(size_t)k] = end[(size_t)k];
        if (all_eof) planned_all = true;
        return true;
      };
      // a round's slices by value: `rounds` grows (and reallocates) on this thread while earlier rounds merge
      auto prep = [&](size_t q, std::vector<std::pair<int64_t, int64_t>> rr, std::vector<uint8_t*> mems) {
        if (hipSetDevice(device) != hipSuccess) throw UdaError("hipSetDevice failed");
        std::vector<Span> views((size_t)K);
        for (int k = 0; k < K; ++k)
          views[(size_t)k] = Span{mems[(size_t)k] + rr[(size_t)k].first, rr[(size_t)k].second - rr[(size_t)k].first};
        return device_merge(*wsv[q % 3], views, Codec::kNone, kind_, kv, sv[q % 3], nullptr, true);
      };
      std::vector<std::future<DeviceMergeOut>> next;
      // at most three rounds in flight (one delivering, two preparing): workspace q % 3 is free again
      // once round q - 3 has been delivered
      auto issue = [&](size_t q) {
        while (next.size() < rounds.size() && next.size() < q + 3) {
          std::vector<uint8_t*> mems((size_t)K);
          for (int k = 0; k < K; ++k) mems[(size_t)k] = runs[(size_t)k].mem;
          next.push_back(std::async(std::launch::async, prep, next.size(), rounds[next.size()], std::move(mems)));
        }
      };
      size_t q = 0;
      while (!planned_all || q < rounds.size()) {
        // plan what has arrived (wait only when nothing is queued)
        while (!planned_all && (q + 2 >= rounds.size())) {
          const size_t before = rounds.size();
          if (!plan_more(q >= rounds.size())) break;
          if (rounds.size() == before && q < rounds.size()) break;
        }
        issue(q);
        if (q >= rounds.size()) continue;
        DeviceMergeOut m = next[q].get();
        issue(q);
        deliver(m, planned_all && q + 1 == rounds.size(), sv[q % 3], *wsv[q % 3]);
        ++q;
      }
      for (auto& t : dp.threads) t.join();
      prog_fetch_ms = std::chrono::duration<double, std::milli>(dp.t_end - t0).count();
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.rpq_rounds = (int64_t)rounds.size();
      }
      for (int k = 0; k < K; ++k) {
        progress_count_++;
        total_count_++;
        {
          std::lock_guard<std::mutex> gl(st_mu_);
          st_.maps_fetched++;
        }
        if (progress_count_ == 20 || total_count_ == maps) {
          host_->fetch_over();
          progress_count_ = 0;
        }
      }
    } else if (progressive) {
      ProgFetch& pf = *prog;
      const int K = pf.K;
      std::vector<int64_t> start((size_t)K, 0), land((size_t)K, 0);
      for (int p = 0; p < pf.P; ++p) {
        const auto tw = std::chrono::steady_clock::now();
        {
          std::unique_lock<std::mutex> lk(pf.mu);
          // exit() sets stop_ without notifying pf.cv: wake up to look
          while (!pf.cv.wait_for(lk, std::chrono::milliseconds(50),
                                 [&] { return pf.done[(size_t)p] == K || pf.err || stop_; })) {
          }
          if (pf.err) std::rethrow_exception(pf.err);
          if (stop_) throw UdaError("reduce task stopped during fetch");
          for (int k = 0; k < K; ++k) land[(size_t)k] = std::max(land[(size_t)k], pf.landed[(size_t)p][(size_t)k]);
        }
        stager->flush_group(p);
        ws.h2d_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
        const bool last_phase = p + 1 == pf.P;
        std::vector<Span> spans((size_t)K);
        if (!last_phase) {
          std::vector<const uint8_t*> win((size_t)K);
          std::vector<int64_t> avail((size_t)K);
          std::vector<char> fin((size_t)K);
          for (int k = 0; k < K; ++k) {
            win[(size_t)k] = pf.dev[(size_t)k] + start[(size_t)k];
            avail[(size_t)k] = land[(size_t)k] - start[(size_t)k];
            fin[(size_t)k] = land[(size_t)k] >= pf.cap[(size_t)k];
          }
          const auto tp = std::chrono::steady_clock::now();
          const gpu::ProgressiveSplit sp = gpu::plan_progressive_split(win, avail, fin, (int)kind_, ws.rounds, s);
          ws.device_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
          int64_t take = 0;
          for (int k = 0; k < K; ++k) take += sp.split[(size_t)k];
          if (take == 0) continue;  // nothing complete below the bound yet: wait for the next phase
          for (int k = 0; k < K; ++k) {
            spans[(size_t)k] = Span{pf.dst[(size_t)k] + start[(size_t)k], sp.split[(size_t)k],
                                    pf.dev[(size_t)k] + start[(size_t)k]};
            start[(size_t)k] += sp.split[(size_t)k];
          }
          {
            std::lock_guard<std::mutex> g(st_mu_);
            st_.rpq_rounds++;  // progressive phases merged
          }
        } else {
          prog_fetch_ms = std::chrono::duration<double, std::milli>(pf.t_end - t0).count();
          for (int k = 0; k < K; ++k)
            spans[(size_t)k] = Span{pf.dst[(size_t)k] + start[(size_t)k], pf.cap[(size_t)k] - start[(size_t)k],
                                    pf.dev[(size_t)k] + start[(size_t)k]};
        }
        device_merge(ws, spans, Codec::kNone, kind_, kv, s,
                     [&](const std::vector<int64_t>& cuts, int64_t records, bool last) {
                       DeviceMergeOut r;
                       r.cuts = cuts;
                       r.records = records;
                       deliver(r, last && last_phase, ws.copy_stream(), ws);
                     });
      }
      for (auto& t : pf.threads) t.join();
      for (int k = 0; k < K; ++k) {
        progress_count_++;
        total_count_++;
        {
          std::lock_guard<std::mutex> gl(st_mu_);
          st_.maps_fetched++;
        }
        if (progress_count_ == 20 || total_count_ == maps) {
          host_->fetch_over();
          progress_count_ = 0;
        }
      }
    } else if (spills.empty() && !direct) {
      // ---- online: the whole reduce input in one device merge
      if (stager) {
        const auto tf = std::chrono::steady_clock::now();
        stager->flush();
        ws.h2d_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf).count();
      }
      // rounds of the merged output go out on the copy stream while the next round merges
      DeviceMergeOut m = device_merge(ws, group, stage_codec, kind_, kv, s,
                                      [&](const std::vector<int64_t>& cuts, int64_t records, bool last) {
                                        DeviceMergeOut r;
                                        r.cuts = cuts;
                                        r.records = records;
                                        deliver(r, last, ws.copy_stream(), ws);
                                      });
      count_decoded(m.decoded_blocks);
    } else {
      // ---- hybrid: last LPQ, then RPQ rounds over the spilled runs (direct: over the partitions)
      if (direct) {
        spills = direct_head.get();
        for (auto& r : direct_runs) spills.push_back(std::move(r));
      } else {
        spill_group();
        lpq_wait();
      }
      const int R = (int)spills.size();
      struct Sample {
        int run;
        int idx;
      };
      std::vector<Sample> samples;
      for (int r = 0; r < R; ++r)
        for (int j = 0; j < (int)spills[(size_t)r].cut.size(); ++j) samples.push_back({r, j});
      std::stable_sort(samples.begin(), samples.end(), [&](const Sample& a, const Sample& b) {
        const int c = cmp_key(kind_, spills[(size_t)a.run].key[(size_t)a.idx], spills[(size_t)b.run].key[(size_t)b.idx]);
        return c != 0 ? c < 0 : (a.run != b.run ? a.run < b.run : a.idx < b.idx);
      });
      // splitters every ~budget/2 bytes of input (a sample stands for the bytes up to its run's next cut)
      const int64_t target = std::max<int64_t>(budget / 2, kSampleSpacing);
      std::vector<std::string> split;
      int64_t acc = 0;
      for (const Sample& sm : samples) {
        const SpillRun& run = spills[(size_t)sm.run];
        const int64_t next = (size_t)sm.idx + 1 < run.cut.size() ? run.cut[(size_t)sm.idx + 1] : run.bytes;
        if (acc >= target) {
          const std::string& k = run.key[(size_t)sm.idx];
          if (split.empty() || cmp_key(kind_, split.back(), k) < 0) {
            split.push_back(k);
            acc = 0;
          }
        }
        acc += next - run.cut[(size_t)sm.idx];
      }
      // read [off, off+len) of a spilled run into dst
      auto read_run = [&](const SpillRun& run, int64_t off, int64_t len, uint8_t* dst) {
        if (len <= 0) return;
        if (run.fd < 0) {
          std::memcpy(dst, run.mem + off, (size_t)len);
          return;
        }
        std::atomic<int64_t> err{0};
        constexpr int64_t kPiece = 8 << 20;
        for (int64_t o = 0; o < len; o += kPiece)
          aio->read(run.fd, off + o, std::min(kPiece, len - o), dst + o, [&err](int64_t r) {
            if (r < 0) err = r;
          });
        aio->drain();
        if (err.load() < 0) throw UdaError("spill read failed");
      };
      // boundary of run r for splitter k: first record whose key >= k
      auto boundary = [&](const SpillRun& run, const std::string& k) -> int64_t {
        // last cut with key < k (cut keys ascend within a run)
        int lo = -1, hi = (int)run.cut.size();
        while (hi - lo > 1) {
          const int mid = (lo + hi) / 2;
          if (cmp_key(kind_, run.key[(size_t)mid], k) < 0)
            lo = mid;
          else
            hi = mid;
        }
        if (lo < 0) return 0;
        const int64_t b = run.cut[(size_t)lo];
        const int64_t e = (size_t)lo + 1 < run.cut.size() ? run.cut[(size_t)lo + 1] : run.bytes;
        std::vector<uint8_t> win;
        const uint8_t* w = run.mem ? run.mem + b : nullptr;  // DRAM runs are scanned in place
        if (!w) {
          win.resize((size_t)(e - b));
          read_run(run, b, e - b, win.data());
          w = win.data();
        }
        int64_t p = 0;
        while (b + p < e) {
          RecordView rv;
          if (ifile_parse(w + p, (size_t)(e - b - p), &rv) != Parse::kRecord)
            throw UdaError("spill scan: bad record");
          if (key_compare(kind_, rv.key, rv.klen, reinterpret_cast<const uint8_t*>(k.data()), (int)k.size()) >= 0)
            break;
          p += rv.size();
        }
        return b + p;
      };
      std::vector<std::vector<int64_t>> bnd((size_t)R);
      auto run_bounds = [&](int r) {
        bnd[(size_t)r].push_back(0);
        for (auto& k : split) bnd[(size_t)r].push_back(boundary(spills[(size_t)r], k));
        bnd[(size_t)r].push_back(spills[(size_t)r].bytes);
      };
      bool all_mem = true;
      for (const SpillRun& run : spills) all_mem = all_mem && run.fd < 0;
      if (all_mem && R > 1) {  // in-place scans of DRAM runs, spread over threads (files share one AsyncIO)
        std::atomic<int> nr{0};
        std::vector<std::exception_ptr> errs((size_t)R);
        std::vector<std::thread> ts;
        for (int w = 0; w < std::min(R, 8); ++w)
          ts.emplace_back([&] {
            for (int r; (r = nr++) < R;) try {
                run_bounds(r);
              } catch (...) {
                errs[(size_t)r] = std::current_exception();
              }
          });
        for (auto& t : ts) t.join();
        for (auto& e : errs)
          if (e) std::rethrow_exception(e);
      } else {
        for (int r = 0; r < R; ++r) run_bounds(r);
      }
      const int rounds = (int)split.size() + 1;
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.rpq_rounds = rounds;
      }
      // RPQ rounds: each round's slices are read, copied to HBM and merged on a helper thread (its own
      // workspace and stream) while earlier rounds are delivered.
      ws2_lease.obj = DevicePool<DeviceWorkspace>::get().acquire(device, [] { return std::make_unique<DeviceWorkspace>(); });
      ws2 = ws2_lease.obj.get();
      ws2->reset_stats();
      // Three workspaces, two rounds prepared ahead: round q + 2's slices cross PCIe (SDMA H2D) while
      // round q + 1 merges and round q is delivered (D2H), so the rounds cost max(H2D, merge, D2H)
      // each instead of H2D + merge.
      ws3_lease.obj = DevicePool<DeviceWorkspace>::get().acquire(device, [] { return std::make_unique<DeviceWorkspace>(); });
      ws3 = ws3_lease.obj.get();
      ws3->reset_stats();
      StreamGuard sg2, sg3;
      sg2.s = gpu::pooled_stream();
      sg3.s = gpu::pooled_stream();
      DeviceWorkspace* wsv[3] = {&ws, ws2, ws3};
      hipStream_t sv[3] = {s, sg2.s, sg3.s};
      gpu::PinnedArena slice_mem[3];
      auto prep = [&](int q) {
        if (hipSetDevice(device) != hipSuccess) throw UdaError("hipSetDevice failed");
        std::vector<Span> views;
        gpu::PinnedArena& sm = slice_mem[q % 3];
        sm.release_all();  // round q - 3's slices: copied to HBM before its merge returned
        for (int r = 0; r < R; ++r) {
          const SpillRun& run = spills[(size_t)r];
          const int64_t b = bnd[(size_t)r][(size_t)q], e = bnd[(size_t)r][(size_t)q + 1];
          if (run.fd < 0) {
            views.push_back(Span{run.mem + b, e - b});
          } else {
            uint8_t* p = sm.alloc((size_t)std::max<int64_t>(e - b, 1));
            read_run(run, b, e - b, p);
            views.push_back(Span{p, e - b});
          }
        }
        // views: pinned host spans (spill arena or slice arena): SDMA H2D, not a blit kernel
        return device_merge(*wsv[q % 3], views, Codec::kNone, kind_, kv, sv[q % 3], nullptr, true);
      };
      std::vector<std::future<DeviceMergeOut>> next((size_t)rounds);
      for (int q = 0; q < std::min(rounds, 2); ++q) next[(size_t)q] = std::async(std::launch::async, prep, q);
      for (int q = 0; q < rounds; ++q) {
        DeviceMergeOut m = next[(size_t)q].get();
        // workspace (q + 2) % 3 delivered round q - 1 before this iteration
        if (q + 2 < rounds) next[(size_t)q + 2] = std::async(std::launch::async, prep, q + 2);
        const int64_t td = trace::host_enabled() ? trace::now_ns() : 0;
        deliver(m, q + 1 == rounds, sv[q % 3], *wsv[q % 3]);
        if (td) trace::host_event("rpq_deliver", m.bytes, q, td, trace::now_ns());
      }
    }
    if (!eof_sent) {  // empty final round (or empty input): EOF alone
      const uint8_t eof[2] = {0xFF, 0xFF};
      if (host_->data_from_uda(eof, kEofBytes) != 0) throw UdaError("dataFromUda callback failed");
      std::lock_guard<std::mutex> g(st_mu_);
      st_.buffers++;
      st_.bytes_delivered += kEofBytes;
    }
    cleanup(true);
    HIP_CHECK(hipStreamSynchronize(s));
    ws_lease.clean = true;
    ws2_lease.clean = true;
    ws3_lease.clean = true;
    stager_lease.clean = true;
    stager_lease2.clean = true;
    std::lock_guard<std::mutex> g(st_mu_);
    st_.gpu_h2d_ms = ws.h2d_ms + (ws2 ? ws2->h2d_ms : 0) + (ws3 ? ws3->h2d_ms : 0);
    st_.gpu_device_ms = ws.device_ms + (ws2 ? ws2->device_ms : 0) + (ws3 ? ws3->device_ms : 0);
    st_.gpu_d2h_wait_ms = ws.d2h_ms + (ws2 ? ws2->d2h_ms : 0) + (ws3 ? ws3->d2h_ms : 0);
    st_.gpu_sink_ms = ws.sink_ms + (ws2 ? ws2->sink_ms : 0) + (ws3 ? ws3->sink_ms : 0);
    st_.fetch_ms = prog_fetch_ms >= 0 ? prog_fetch_ms : fetch_ms;
    st_.merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - st_.fetch_ms;
    if (trace::host_enabled()) {
      trace::host_event("task", stage_step, drains,
                        trace::now_ns() - (int64_t)((st_.merge_ms + fetch_ms) * 1e6), trace::now_ns());
      trace::host_dump();
    }
  } catch (...) {
    if (lpq_thr.joinable()) lpq_thr.join();  // the LPQ thread uses this frame's state
    cleanup(false);
    throw;
  }
}

// The partitions a device-fetch task gets no usable descriptor for (the provider's HBM store is full or
// off, or the descriptor cannot be mapped here). Two sources:
//  * the MOF file itself, when the provider runs on this node and named the file in its answer, and the
//    file is a regular file of this process's user (mapred.uda.gpu.fetch.local.read, default on; never for
//    a confined task): pread into pinned slots, one copy out of the page cache;
//  * otherwise the provider, over the transport: three requests of `chunk` bytes in flight per worker.
// `streams` workers (mapred.uda.gpu.fetch.bytes.streams, default 4) take partitions in turn; every landed
// chunk goes on to the device (H2D on the worker's stream) while the next ones come in. The round-5 loop
// had one request of the task's buffer size (1 MiB) in flight at a time: a round trip per MiB, 3.3 GB/s
// per task, 19.6 GB/s for a node of 15 tasks with 42.9 GB of 62.4 GB declined per wave; pipelined TCP
// 24.0 (profiles/r6/r6j_*, r6k_nodefiles62_store20.log). Over TCP every byte is copied twice by the CPU
// (the provider's sendfile, the reducer's receive) next to the consumers' own copies. The reference's
// fetcher keeps its requests in flight the same way (Segment::send_request, src/Merger/StreamRW.cc).
bool mof_host_is_local(const std::string& spec) {
  std::string h = spec;
  if (const size_t c = h.rfind(':'); c != std::string::npos && h.find(':') == c) h = h.substr(0, c);
  if (h == "127.0.0.1" || h == "localhost" || h == "::1" || h.empty()) return true;
  char me[256] = {0};
  if (::gethostname(me, sizeof(me) - 1) != 0) return false;
  const std::string m = me;
  return h == m || h == m.substr(0, m.find('.')) || m == h.substr(0, h.find('.'));
}

int open_local_mof(const std::string& path, int64_t off, int64_t len) {
  if (path.empty() || path[0] != '/') return -1;
  const int fd = ::open(path.c_str(), O_RDONLY | O_NOFOLLOW | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat sb;
  if (::fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_uid != ::geteuid() || sb.st_size < off + len) {
    ::close(fd);
    return -1;
  }
  return fd;
}

int64_t ReduceTask::fetch_declined_bytes(int device, const std::vector<DeclinedPart>& parts, gpu::DeviceBuffer& dst,
                                         std::vector<const uint8_t*>* where, int64_t* local) {
  const size_t n = parts.size();
  std::vector<int64_t> at(n + 1, 0);
  for (size_t k = 0; k < n; ++k) at[k + 1] = at[k] + ((parts[k].len + 255) & ~(int64_t)255);
  DeviceWorkspace::ensure(dst, at[n]);
  uint8_t* base = dst.as<uint8_t>();
  where->assign(n, nullptr);
  for (size_t k = 0; k < n; ++k) (*where)[k] = base + at[k];
  const int streams = (int)std::clamp<int64_t>(host_->conf_i64("mapred.uda.gpu.fetch.bytes.streams", 4), 1, 16);
  int64_t chunk = std::max<int64_t>(buffer_size_, host_->conf_i64("mapred.uda.gpu.fetch.bytes.chunk", 8ll << 20));
  chunk = (chunk + 4095) & ~(int64_t)4095;
  const bool local_ok = !sandbox_.enabled && host_->conf_i64("mapred.uda.gpu.fetch.local.read", 1) != 0;
  constexpr int kSlots = 3;
  std::atomic<size_t> next{0};
  std::atomic<int64_t> fetched{0}, read_here{0};
  std::mutex em;
  std::string err;
  auto failed = [&] {
    std::lock_guard<std::mutex> g(em);
    return !err.empty();
  };
  auto worker = [&] {
    struct Slot {
      gpu::PinnedPool::Block b;
      hipEvent_t ev = nullptr;
      bool h2d = false;   // an H2D from this slot may still be reading it
      bool busy = false;  // a request into this slot is in flight
      bool done = false;
      int64_t off = 0, want = 0;
      FetchAck a;
    };
    Slot sl[kSlots];
    std::mutex m;
    std::condition_variable cv;
    hipStream_t hs = nullptr;
    int fd = -1;
    auto drain = [&] {  // every request answered (their callbacks touch sl), every H2D done
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] {
        for (auto& x : sl)
          if (x.busy && !x.done) return false;
        return true;
      });
      lk.unlock();
      if (hs) (void)hipStreamSynchronize(hs);
    };
    auto reuse = [&](Slot& x) {  // the slot's previous H2D has read it
      if (x.h2d) {
        HIP_CHECK(hipEventSynchronize(x.ev));
        x.h2d = false;
      }
    };
    auto to_device = [&](Slot& x, uint8_t* dev) {
      HIP_CHECK(hipMemcpyAsync(dev + x.off, x.b.p, (size_t)x.want, hipMemcpyHostToDevice, hs));
      HIP_CHECK(hipEventRecord(x.ev, hs));
      x.h2d = true;
      fetched += x.want;
    };
    try {
      HIP_CHECK(hipSetDevice(device));
      hs = gpu::pooled_stream();
      for (auto& x : sl) {
        x.b = gpu::PinnedPool::instance().acquire((size_t)chunk);
        HIP_CHECK(hipEventCreateWithFlags(&x.ev, hipEventDisableTiming));
      }
      for (;;) {
        const size_t k = next.fetch_add(1);
        if (k >= n || failed() || stop_) break;
        const DeclinedPart& d = parts[k];
        const FetchParams& f = d.f;
        const int64_t L = d.len;
        uint8_t* dev = base + at[k];
        fd = local_ok && mof_host_is_local(f.host) ? open_local_mof(d.path, d.file_off, L) : -1;
        if (fd >= 0) {
          for (int64_t off = 0, s = 0; off < L; s = (s + 1) % kSlots) {
            Slot& x = sl[s];
            reuse(x);
            x.off = off;
            x.want = std::min(chunk, L - off);
            for (int64_t got = 0; got < x.want;) {
              const ssize_t r = ::pread(fd, x.b.p + got, (size_t)(x.want - got), (off_t)(d.file_off + off + got));
              if (r < 0 && errno == EINTR) continue;
              if (r <= 0)
                throw UdaError("reading " + d.path + " for " + f.map_id + ": " + (r < 0 ? strerror(errno) : "short file"));
              got += r;
            }
            to_device(x, dev);
            read_here += x.want;
            off += x.want;
          }
          ::close(fd);
          fd = -1;
          continue;
        }
        int64_t issue_off = 0;
        int outstanding = 0, head = 0, tail = 0;  // slots in request order: tail (oldest) .. head
        auto issue = [&](int s) {
          Slot& x = sl[s];
          reuse(x);
          FetchRequest req;
          req.job_id = f.job_id;
          req.map_id = f.map_id;
          req.reduce_id = f.reduce_id;
          req.fetched = issue_off;
          req.buf_len = chunk;
          {
            std::lock_guard<std::mutex> g(m);
            x.busy = true;
            x.done = false;
            x.off = issue_off;
            x.want = std::min(chunk, L - issue_off);
          }
          issue_off += x.want;
          ++outstanding;
          fetch_begin();
          transport_->fetch(f.host, req, x.b.p, [&, s](const FetchAck& a) {
            {
              // notify under the lock: once drain() sees every answer the worker's frame (m, cv) goes away
              std::lock_guard<std::mutex> g(m);
              sl[s].a = a;
              sl[s].done = true;
              cv.notify_all();
            }
            fetch_end();
          });
        };
        while (outstanding < kSlots && issue_off < L) {
          issue(head);
          head = (head + 1) % kSlots;
        }
        while (outstanding > 0) {
          Slot& x = sl[tail];
          {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return x.done; });
            x.busy = false;
          }
          --outstanding;
          if (x.a.status != 0) throw UdaError("fetch of " + f.map_id + " failed: " + x.a.error);
          if (x.a.sent != x.want || x.a.part_len != L)
            throw UdaError("fetch of " + f.map_id + ": provider sent " + std::to_string(x.a.sent) + " bytes of a " +
                           std::to_string(x.a.part_len) + "-byte partition at offset " + std::to_string(x.off) +
                           " (expected " + std::to_string(x.want) + " of " + std::to_string(L) + ")");
          to_device(x, dev);
          tail = (tail + 1) % kSlots;
          if (issue_off < L) {
            issue(head);
            head = (head + 1) % kSlots;
          }
        }
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(em);
      if (err.empty()) err = e.what();
    }
    if (fd >= 0) ::close(fd);
    drain();
    for (auto& x : sl) {
      if (x.ev) (void)hipEventDestroy(x.ev);
      if (x.b.p) gpu::PinnedPool::instance().release(x.b);
    }
    if (hs) gpu::return_stream(hs);
  };
  std::vector<std::thread> ts;
  const int nw = (int)std::min<size_t>((size_t)streams, n);
  for (int i = 1; i < nw; ++i) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  if (!err.empty()) throw UdaError(err);
  if (stop_) throw UdaError("reduce task stopped during fetch");
  *local = read_here.load();
  return fetched.load();
}

// GPU backend, device fetch (mapred.uda.gpu.fetch=device, uncompressed map outputs): every FETCH is
// a descriptor fetch, so partitions the provider holds in HBM are merged where they live (same
// process: the address; another process on the node: an IPC mapping) and never cross PCIe on the
// way in. MOFs that are not device-resident are fetched as bytes and copied to the device.
// TeraSort-shaped inputs go through the key-range-round FIXED10 merge with SDMA delivery
// (device_reduce.cc); other key classes through the generic merge tree.
// Reference: start_fetch_req / RDMA WRITE into the reducer buffer (src/DataNet/RDMAClient.cc:559-600,
// src/DataNet/RDMAServer.cc:537-631) and merge_online (src/Merger/MergeManager.cc:184-193).
bool ReduceTask::merge_gpu_device(bool probe) {
  join_prewarm();
  if (gpu::device_count() <= 0) throw UdaError("mapred.uda.merge.backend=gpu but no HIP device is visible");
  // The task's device memory mostly comes from pooled workspaces sized by earlier tasks, so a
  // DeviceBuffer allocation may never happen in this task: the injected device-allocation failure
  // (UDA_FAULT_DEVICE_ALLOC) also counts the task taking its workspaces.
  if (fault_hit("DEVICE_ALLOC")) throw UdaError("injected device allocation failure (GPU merge workspaces)");
  auto t0 = std::chrono::steady_clock::now();
  auto boot_ms = [] {
    timespec ts{};
    clock_gettime(CLOCK_BOOTTIME, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6;
  };
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.merge_start_boot_ms = boot_ms();
  }
  const int maps = init_.num_maps;
  const int device = device_;
  HIP_CHECK(hipSetDevice(device));
  HIP_PENDING("the device fetch");
  StreamGuard sg;
  sg.s = gpu::pooled_stream();
  hipStream_t s = sg.s;
  // Descriptors are references the providers keep for this task (gpu/mof_cache.h): released when the
  // task is done with them -- its merge finished, or it failed -- after the device has stopped
  // reading the partitions (the merge stream is synchronized first).
  const std::string holder = gpu::reducer_holder_id(init_.reduce_task_id);
  struct DescRelease {
    ReduceTask* t;
    StreamGuard& sg;
    const std::string& holder;
    std::vector<std::string> descs;
    std::set<std::string> hosts;
    ~DescRelease() {
      if (sg.s) (void)hipStreamSynchronize(sg.s);
      for (const auto& d : descs) gpu::release_device_descriptor(d);
      try {
        t->release_descriptors(hosts, holder);
      } catch (const std::exception& e) {
        UDA_LOG(kWarn, "releasing descriptors: %s", e.what());
      }
    }
  } desc_release{this, sg, holder, {}, {}};
  struct Part {
    const uint8_t* dptr = nullptr;
    int64_t part_len = 0;
  };
  std::vector<std::unique_ptr<Part>> parts;
  int64_t host_bytes = 0, descriptors = 0, unmapped = 0;
  // partitions answered "not device-resident" (or with a descriptor this process cannot map): their
  // bytes are fetched once every descriptor answer is in (fetch_declined, below)
  std::vector<DeclinedPart> declined;
  std::vector<size_t> declined_part;  // index into parts

  // ---- fetch phase: descriptors for every MOF as its FETCH arrives
  int resolved = 0;
  while (resolved < maps) {
    std::vector<FetchParams> batch;
    const auto tw = std::chrono::steady_clock::now();
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !fetch_list_.empty(); });
      if (stop_) throw UdaError("reduce task stopped during fetch");
      while (!fetch_list_.empty()) {
        batch.push_back(fetch_list_.front());
        fetch_list_.pop_front();
      }
    }
    const auto ta = std::chrono::steady_clock::now();
    if (resolved == 0) {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.fetch_sent_boot_ms = boot_ms();
    }
    std::vector<FetchAck> acks(batch.size());
    std::mutex m;
    std::condition_variable c;
    size_t left = batch.size();
    for (size_t i = 0; i < batch.size(); ++i) {
      FetchRequest req;
      req.job_id = batch[i].job_id;
      req.map_id = batch[i].map_id;
      req.reduce_id = batch[i].reduce_id;
      req.buf_len = kDescriptorFetch;
      req.holder = holder;
      desc_release.hosts.insert(batch[i].host);
      fetch_begin();
      transport_->fetch(batch[i].host, req, nullptr, [&, i](const FetchAck& a) {
        std::lock_guard<std::mutex> g(m);
        acks[i] = a;
        --left;
        c.notify_all();
        fetch_end();
      });
    }
    {
      std::unique_lock<std::mutex> lk(m);
      c.wait(lk, [&] { return left == 0; });
    }
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.fetch_cmd_wait_ms += std::chrono::duration<double, std::milli>(ta - tw).count();
      st_.fetch_ack_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count();
    }
    if (probe && resolved == 0 && descriptors == 0) {
      // auto mode: the first answers decide; host-resident map outputs keep the staged path
      bool any_device = false;
      for (const auto& a : acks) any_device |= a.status == 0 && gpu::is_device_descriptor(a.path);
      if (!any_device) {
        std::lock_guard<std::mutex> g(mu_);
        for (auto it = batch.rbegin(); it != batch.rend(); ++it) fetch_list_.push_front(*it);
        return false;
      }
    }
    for (size_t i = 0; i < batch.size(); ++i) {
      const FetchAck& a = acks[i];
      auto part = std::make_unique<Part>();
      std::string why;
      const uint8_t* dp = nullptr;
      const auto tm = std::chrono::steady_clock::now();
      if (a.status == 0 && gpu::is_device_descriptor(a.path)) {
        dp = gpu::try_resolve_device_descriptor(a.path, device, &why);
        std::lock_guard<std::mutex> g(st_mu_);
        st_.descriptor_map_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tm).count();
      }
      if (dp != nullptr) {
        part->dptr = dp;
        part->part_len = a.part_len;
        desc_release.descs.push_back(a.path);
        ++descriptors;
      } else if (a.status == 0 && gpu::is_device_descriptor(a.path)) {
        // not mappable here (another node, no IPC handle, import failure): fetch its bytes
        UDA_LOG(kInfo, "descriptor of %s not usable (%s): fetching bytes", batch[i].map_id.c_str(), why.c_str());
        if (unmapped == 0) {
          std::lock_guard<std::mutex> g(st_mu_);
          st_.unmapped_reason = why;
        }
        if (a.part_len < kEofBytes)
          throw UdaError("fetch of " + batch[i].map_id + ": descriptor answer carries no partition length");
        part->part_len = a.part_len;
        declined.push_back(DeclinedPart{batch[i], a.part_len, std::string(), 0});
        declined_part.push_back(parts.size());
        ++unmapped;
      } else if (a.status == kNotDeviceResident) {
        // every partition holds at least the IFile EOF marker: a length of 0 is a provider that did not say
        if (a.part_len < kEofBytes)
          throw UdaError("fetch of " + batch[i].map_id + ": declined descriptor fetch carries no partition length (" +
                         std::to_string(a.part_len) + ")");
        part->part_len = a.part_len;
        declined.push_back(DeclinedPart{batch[i], a.part_len, a.path, a.mof_offset});
        declined_part.push_back(parts.size());
      } else {
        throw UdaError("fetch of " + batch[i].map_id + " failed: " + (a.status ? a.error : "no device descriptor"));
      }
      parts.push_back(std::move(part));
      resolved++;
      progress_count_++;
      total_count_++;
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.maps_fetched++;
        st_.bytes_fetched += parts.back()->part_len;
      }
      if (progress_count_ == 20 || total_count_ == maps) {
        host_->fetch_over();
        progress_count_ = 0;
      }
    }
  }
  double fetch_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  HIP_PENDING("the end of the descriptor fetch");
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.device_descriptors = descriptors;
    st_.unmapped_descriptors = unmapped;
  }

  auto sink = [&](const uint8_t* p, int64_t len) -> int {
    if (stop_) throw UdaError("reduce task stopped during merge");
    const int r = host_->data_from_uda(p, (int32_t)len);
    std::lock_guard<std::mutex> g(st_mu_);
    if (st_.buffers == 0)
      st_.first_data_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st_.buffers++;
    st_.bytes_delivered += len;
    return r;
  };
  int64_t in_bytes = 0;
  for (const auto& p : parts) in_bytes += p->part_len;
  PoolLease<DeviceWorkspace> ws_lease{device, DevicePool<DeviceWorkspace>::get().acquire_fit(
                                                  device, in_bytes, [] { return std::make_unique<DeviceWorkspace>(); })};
  DeviceWorkspace& ws = *ws_lease.obj;
  ws.reset_stats();
  HIP_PENDING("the merge workspace");
  int64_t local_bytes = 0;
  if (!declined.empty()) {
    const auto tf = std::chrono::steady_clock::now();
    // the node's tasks take turns (FIFO, mapred.uda.gpu.fetch.bytes.slots at once; 0 = no limit): served
    // in turn, the first tasks' bytes are in and their merges deliver while later tasks still fetch;
    // all at once, every task's bytes landed late together and the link idled until then
    GateLease bgate;
    bgate.which = 2;
    if (const int slots = (int)host_->conf_i64("mapred.uda.gpu.fetch.bytes.slots", 4); slots > 0) {
      if (!DeviceGate::get(2).acquire(device, slots, [&] { return stop_.load(); }))
        throw UdaError("reduce task stopped while waiting for its turn to fetch bytes");
      bgate.device = device;
    }
    const double tg = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf).count();
    std::vector<const uint8_t*> where;
    host_bytes = fetch_declined_bytes(device, declined, ws.fetched, &where, &local_bytes);
    for (size_t k = 0; k < declined.size(); ++k) parts[declined_part[k]]->dptr = where[k];
    fetch_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf).count();
    std::lock_guard<std::mutex> g(st_mu_);
    st_.gpu_gate_wait_ms += tg;
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.host_fetched_bytes = host_bytes;
    st_.local_read_bytes = local_bytes;
  }
  // HBM admission (gpu/hbm_ledger.h): the task's device working set -- decoded partitions, the
  // key-range round's output slots and merge tables -- is reserved before it is allocated, under the
  // device's byte budget shared with the provider's store and every other task on the node. A round
  // that could never fit is halved until it does; a task that fits later waits (FIFO) for it.
  gpu::HbmLedger& ledger = gpu::HbmLedger::get();
  std::unique_ptr<gpu::HbmLedger::Reservation> hbm_res;
  int64_t round_bytes = host_->conf_i64("mapred.uda.gpu.round.bytes", 2ll << 30);
  auto admit = [&](int64_t fixed, const std::function<int64_t(int64_t)>& round_ws) {
    const int64_t hr = ledger.headroom(device);
    while (round_bytes > (64ll << 20) && fixed + round_ws(round_bytes) > hr) round_bytes /= 2;
    hbm_res = ledger.reserve(device, std::max<int64_t>(0, fixed + round_ws(round_bytes)), [&] { return stop_.load(); });
    std::lock_guard<std::mutex> g(st_mu_);
    st_.hbm_wait_ms += hbm_res->wait_ms();
    st_.hbm_reserved = hbm_res->granted();
    st_.round_bytes = round_bytes;
  };
  // ---- compressed map outputs: F6 block decode straight from the partitions (descriptors or fetched
  // bytes) into the workspace; the framing is walked on the device
  if (codec_ != Codec::kNone) {
    const auto td = std::chrono::steady_clock::now();
    std::vector<const uint8_t*> cp;
    std::vector<int64_t> cl;
    for (const auto& p : parts) {
      cp.push_back(p->dptr);
      cl.push_back(p->part_len);
    }
    gpu::BlockPlan bp;
    std::vector<int64_t> roff;
    int64_t blocks = 0;
    const bool dev_frames = gpu::plan_block_streams_device(codec_, cp, cl, &bp, ws.frame_scratch, ws.frame_descs, s);
    // TeraSort-shaped partitions: decode per key-range round, only the blocks each round covers, so the
    // task's device memory is round-sized instead of its decoded partitions (DecompressorWrapper decodes
    // block by block next to the merge too, src/Merger/DecompressorWrapper.cc:85-114)
    if (dev_frames && kind_ == KeyKind::kText && host_->conf_i64("mapred.uda.gpu.decode.stream", 1) != 0) {
      gpu::DeviceReduceConfig cfg;
      cfg.device = device;
      cfg.kv_buf_bytes = kv_buf_size_;
      cfg.round_bytes = round_bytes;
      cfg.stop = [&] { return stop_.load(); };
      // the node's tasks take turns for each round's block decode (FIFO, this many at once; 0 = no
      // limit). One round's decode (a wave per 256 KiB block, ~8k blocks) leaves the device idle: 130 GB
      // LZO 38.7 GB/s with one at a time, 45.7 with two, 49.3 with three; Snappy 54.0 / 53.9 / 53.3,
      // link-bound (profiles/r5/r5{j,k,l}_*130*.log)
      if (const int slots = (int)host_->conf_i64("mapred.uda.gpu.decode.stream.slots", 3); slots > 0) {
        cfg.decode_turn = [this, device, slots] {
          return DeviceGate::get(1).acquire(device, slots, [&] { return stop_.load(); });
        };
        cfg.decode_done = [device] { DeviceGate::get(1).release(device); };
      }
      bool streamed = false;
      const gpu::DeviceReduceStats ds = gpu::device_reduce_fixed_blocks(cfg, (int)codec_, bp, sink, &streamed);
      if (streamed) {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.hbm_wait_ms += ds.hbm_wait_ms;
        st_.gpu_gate_wait_ms += ds.decode_wait_ms;
        st_.hbm_reserved = ds.hbm_reserved;
        st_.round_bytes = ds.round_bytes;
        st_.records = ds.records;
        st_.rpq_rounds = ds.rounds;
        st_.device_decoded_blocks += ds.decoded_blocks;
        st_.gpu_device_ms = ds.plan_ms + ds.merge_wait_ms;
        st_.gpu_d2h_wait_ms = ds.d2h_wait_ms;
        st_.gpu_sink_ms = ds.sink_ms;
        st_.fetch_ms = fetch_ms;
        st_.merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - fetch_ms;
        st_.merge_path = "device-fixed10-stream";
        ws_lease.clean = true;
        return true;
      }
    }
    if (dev_frames) {
      // decode output and the merge's rounds at once: a task holding its decoded partitions must
      // not then wait for merge memory behind tasks doing the same
      const int64_t raw = bp.raw_total;
      admit(std::max<int64_t>(0, raw + raw / 8 - (int64_t)ws.in.held()), [&](int64_t rb) {
        return gpu::fixed_round_ws_bytes(std::min(rb, raw), (int)parts.size());
      });
    }
    // Decodes of concurrent tasks take turns (FIFO, mapred.uda.gpu.decode.slots at once, default 1;
    // 0 = no limit): a decode fills the device by itself, so running them in turn costs no decode
    // throughput, and the first tasks reach their merge and D2H delivery while later ones still
    // decode. All at once, every task finished decoding together and PCIe idled until then.
    GateLease dgate;
    dgate.which = 1;
    if (const int slots = (int)host_->conf_i64("mapred.uda.gpu.decode.slots", 1); slots > 0) {
      if (!DeviceGate::get(1).acquire(device, slots, [&] { return stop_.load(); }))
        throw UdaError("reduce task stopped while waiting for a device decode slot");
      dgate.device = device;
    }
    if (dev_frames) {
      DeviceWorkspace::ensure(ws.in, bp.raw_total);
      ws.decoder.decode(codec_, bp, nullptr, ws.in.as<uint8_t>(), s);
      roff = bp.raw_offset;
      blocks = (int64_t)bp.descs.size();
    } else {  // framing that needs a decode (multi-chunk LZO blocks): decode on the host
      UDA_LOG(kInfo, "device decode: framing needs a host decode (%s)", codec_name(codec_));
      std::vector<std::vector<uint8_t>> raws;
      roff.assign(1, 0);
      for (size_t i = 0; i < cp.size(); ++i) {
        std::vector<uint8_t> c((size_t)cl[i]);
        if (cl[i] > 0) HIP_CHECK(hipMemcpy(c.data(), cp[i], (size_t)cl[i], hipMemcpyDefault));
        BlockDecoder dec(codec_);
        dec.feed(c.data(), c.size());
        std::vector<uint8_t> raw, buf(1 << 20);
        for (size_t n; (n = dec.read(buf.data(), buf.size())) > 0;) raw.insert(raw.end(), buf.begin(), buf.begin() + (long)n);
        if (!dec.idle()) throw UdaError("truncated compressed partition");
        roff.push_back(roff.back() + (int64_t)raw.size());
        raws.push_back(std::move(raw));
      }
      DeviceWorkspace::ensure(ws.in, roff.back());
      for (size_t i = 0; i < raws.size(); ++i)
        if (!raws[i].empty())
          HIP_CHECK(hipMemcpy(ws.in.as<uint8_t>() + roff[i], raws[i].data(), raws[i].size(), hipMemcpyHostToDevice));
    }
    for (size_t i = 0; i < parts.size(); ++i) {
      parts[i]->dptr = ws.in.as<uint8_t>() + roff[i];
      parts[i]->part_len = roff[i + 1] - roff[i];
    }
    HIP_CHECK(hipStreamSynchronize(s));  // (the merge below syncs it anyway): decode time on its own
    std::lock_guard<std::mutex> g(st_mu_);
    st_.device_decoded_blocks += blocks;
    st_.gpu_decode_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count();
  }
  // ---- TeraSort-shaped input: FIXED10 rounds straight over the partitions
  bool fixed = kind_ == KeyKind::kText;
  std::vector<gpu::RunDesc> runs;
  for (const auto& p : parts) {
    const int64_t rec_bytes = p->part_len - kEofBytes;
    if (rec_bytes < 0 || rec_bytes % gpu::kTeraRecordBytes != 0) fixed = false;
    gpu::RunDesc d;
    d.base = p->dptr;
    d.nbytes = std::max<int64_t>(rec_bytes, 0);
    d.nrec = d.nbytes / gpu::kTeraRecordBytes;
    d.offsets = nullptr;
    runs.push_back(d);
  }
  if (fixed && gpu::runs_are_fixed10(runs, s)) {
    gpu::DeviceReduceConfig cfg;
    cfg.device = device;
    cfg.kv_buf_bytes = kv_buf_size_;
    cfg.round_bytes = round_bytes;
    cfg.stop = [&] { return stop_.load(); };
    gpu::DeviceReduceStats ds = gpu::device_reduce_fixed(cfg, runs, sink);
    std::lock_guard<std::mutex> g(st_mu_);
    if (!hbm_res) {
      st_.hbm_wait_ms += ds.hbm_wait_ms;
      st_.hbm_reserved = ds.hbm_reserved;
    }
    st_.round_bytes = ds.round_bytes;
    st_.records = ds.records;
    st_.rpq_rounds = ds.rounds;
    st_.gpu_device_ms = ds.plan_ms + ds.merge_wait_ms;
    st_.gpu_d2h_wait_ms = ds.d2h_wait_ms;
    st_.gpu_sink_ms = ds.sink_ms;
    st_.fetch_ms = fetch_ms;
    st_.merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - fetch_ms;
    st_.merge_path = "device-fixed10";
    ws_lease.clean = true;
    return true;
  }
  // ---- any other key class: the generic merge, reading the partitions where they live, in key-range
  // rounds of at most mapred.uda.gpu.round.bytes of input (generic_rounds.h), so the device working
  // set (output + ~80 B/record of merge metadata) is bounded by the round, not by the partition
  int64_t total = 0;
  std::vector<const uint8_t*> rptr;
  std::vector<int64_t> rlen;
  for (const auto& p : parts) {
    rptr.push_back(p->dptr);
    rlen.push_back(p->part_len);
    total += p->part_len;
  }
  // working set of a generic round of rb input bytes: two output slots + ~88 B of merge metadata per
  // record (records of >= 64 B) over what the pooled workspace already holds
  if (!hbm_res) {
    const int64_t have = (int64_t)(ws.out.held() + ws.out2.held()) + ws.merger.workspace_bytes();
    admit(0, [&](int64_t rb) {
      const int64_t b = std::min(rb, total);
      return std::max<int64_t>(0, (int64_t)(2.25 * (double)b + 1.4 * (double)b) - have);
    });
  }
  if (total > round_bytes) {
    // a task holding more than a round (a skewed partition) is the job's long pole: its merge kernels
    // go first when the device is shared with the other tasks' merges
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamSynchronize(s));
    gpu::return_stream(sg.s);
    sg.s = nullptr;
    sg.s = gpu::pooled_stream(hi);
    s = sg.s;
    // and its delivery pieces go over two SDMA engines instead of one: the link is shared per queued copy,
    // so while the other tasks deliver, this one's output keeps a larger share of it
    ws.out_ways = 2;
  }
  const gpu::GenericRoundsPlan rplan = gpu::plan_generic_rounds(rptr, rlen, (int)kind_, round_bytes, ws.rounds, s);
  // Round q merges into outs[q & 1] while a delivery thread streams round q-1 out (D2H pieces +
  // dataFromUda): the consumer's work (the reduce task's bound when one task holds most of the data)
  // never waits for the merge driver, and the merge reuses an output only after its delivery.
  DeviceWorkspace::ensure(ws.out, rplan.max_round_bytes);
  if (rplan.rounds > 1) DeviceWorkspace::ensure(ws.out2, rplan.max_round_bytes);
  gpu::DeviceBuffer* outs[2] = {&ws.out, rplan.rounds > 1 ? &ws.out2 : &ws.out};
  const int64_t kv = kv_buf_size_ - kEofBytes;
  std::vector<uint8_t> tail((size_t)kv_buf_size_ + kEofBytes);
  bool eof_sent = false;
  struct DJob {
    const uint8_t* src;
    std::vector<int64_t> cuts;
    bool last;          // the task's final records: the EOF marker goes after them
    bool end_of_round;  // the key-range round's output is fully handed over after this job
  };
  std::mutex dmu;
  std::condition_variable dcv;
  std::deque<DJob> djobs;
  int delivered = 0;  // key-range rounds fully delivered
  bool dstop = false;
  std::string derr;
  std::thread dthr([&] {
    try {
      bind_thread_to_cpus(gpu::device_consumer_cpus(device));  // the D2H ring and the consumer copies
      HIP_CHECK(hipSetDevice(device));
      for (;;) {
        DJob j;
        {
          const int64_t ti = trace::host_enabled() ? trace::now_ns() : 0;
          std::unique_lock<std::mutex> lk(dmu);
          dcv.wait(lk, [&] { return dstop || !djobs.empty(); });
          if (djobs.empty()) return;
          j = std::move(djobs.front());
          djobs.pop_front();
          if (ti) trace::host_event("gr_idle", (int64_t)(uintptr_t)&ws, 0, ti, trace::now_ns());
        }
        DeviceMergeOut m;
        m.cuts = std::move(j.cuts);
        const size_t nb = m.cuts.size() < 2 ? 0 : m.cuts.size() - 1;
        stream_out(ws, m, ws.copy_stream(), [&](const uint8_t* piece, size_t c0, size_t c1) {
          for (size_t x = c0; x < c1; ++x) {
            const uint8_t* p = piece + (m.cuts[x] - m.cuts[c0]);
            int64_t len = m.cuts[x + 1] - m.cuts[x];
            if (j.last && x + 1 == nb) {
              std::memcpy(tail.data(), p, (size_t)len);
              tail[(size_t)len] = tail[(size_t)len + 1] = 0xFF;
              p = tail.data();
              len += kEofBytes;
              eof_sent = true;
            }
            if (sink(p, len) != 0) throw UdaError("dataFromUda callback failed");
          }
        }, j.src);
        if (j.end_of_round) {
          std::lock_guard<std::mutex> g(dmu);
          ++delivered;
          dcv.notify_all();
        }
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(dmu);
      derr = e.what();
      dstop = true;
      dcv.notify_all();
    }
  });
  struct DJoin {
    std::thread& t;
    std::mutex& mu;
    std::condition_variable& cv;
    bool& stop;
    ~DJoin() {
      {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
      }
      cv.notify_all();
      if (t.joinable()) t.join();
    }
  } djoin{dthr, dmu, dcv, dstop};
  auto push = [&](DJob j) {
    std::lock_guard<std::mutex> g(dmu);
    if (!derr.empty()) throw UdaError("delivery failed: " + derr);
    djobs.push_back(std::move(j));
    dcv.notify_all();
  };
  DeviceMergeOut m;
  for (int q = 0; q < rplan.rounds; ++q) {
    {
      const int64_t tw = trace::host_enabled() ? trace::now_ns() : 0;
      std::unique_lock<std::mutex> lk(dmu);  // outs[q & 1] held round q - 2: delivered?
      dcv.wait(lk, [&] { return delivered >= q - 1 || !derr.empty(); });
      if (!derr.empty()) throw UdaError("delivery failed: " + derr);
      if (tw) trace::host_event("gr_slot_wait", (int64_t)(uintptr_t)&ws, q, tw, trace::now_ns());
    }
    std::vector<const uint8_t*> sp;
    std::vector<int64_t> sl;
    for (size_t k = 0; k < rptr.size(); ++k) {
      const int64_t b = rplan.at((int)k, q), e = rplan.at((int)k, q + 1);
      if (e > b) {
        sp.push_back(rptr[k] + b);
        sl.push_back(e - b);
      }
    }
    const bool last_outer = q + 1 == rplan.rounds;
    if (sp.empty()) {
      push(DJob{nullptr, {}, false, true});
      continue;
    }
    const uint8_t* dst = outs[q & 1]->as<uint8_t>();
    const auto tq = std::chrono::steady_clock::now();
    bool round_closed = false;
    gpu::GenericMergeResult r = ws.merger.merge(
        sp, sl, (int)kind_, outs[q & 1]->as<uint8_t>(), (int64_t)outs[q & 1]->size(), kv, s,
        [&](const std::vector<int64_t>& cuts, int64_t, bool last_inner) {
          push(DJob{dst, cuts, last_inner && last_outer, last_inner});
          round_closed = round_closed || last_inner;
        });
    // slices holding only EOF markers: the merge saw no records and never called back, but the
    // delivery thread still has to count this round as handed over
    if (!round_closed) push(DJob{nullptr, {}, false, true});
    m.records += r.records;
    if (trace::host_enabled())
      trace::host_event("gr_merge", (int64_t)(uintptr_t)&ws, q,
                        trace::now_ns() - (int64_t)(std::chrono::steady_clock::now() - tq).count(), trace::now_ns());
    static const bool trace = std::getenv("UDA_DEVICE_REDUCE_TRACE") != nullptr;  // tools: per-round lines
    if (trace)
      std::fprintf(stderr, "[generic rounds] round %d/%d: %ld records merged in %.1f ms\n", q, rplan.rounds,
                   (long)r.records, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq).count());
  }
  {
    std::unique_lock<std::mutex> lk(dmu);
    dcv.wait(lk, [&] { return delivered >= rplan.rounds || !derr.empty(); });
    if (!derr.empty()) throw UdaError("delivery failed: " + derr);
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.rpq_rounds = rplan.rounds;
    st_.gpu_ws_bytes = (int64_t)ws.out.size() + (rplan.rounds > 1 ? (int64_t)ws.out2.size() : 0) +
                       ws.merger.workspace_bytes();
    st_.gpu_device_ms = rplan.plan_ms;
    st_.gpu_d2h_wait_ms = ws.d2h_ms;
    st_.gpu_sink_ms = ws.sink_ms;
  }
  if (!eof_sent) {
    tail[0] = tail[1] = 0xFF;
    if (sink(tail.data(), kEofBytes) != 0) throw UdaError("dataFromUda callback failed");
  }
  HIP_CHECK(hipStreamSynchronize(s));
  ws_lease.clean = true;
  std::lock_guard<std::mutex> g(st_mu_);
  st_.records = m.records;
  st_.fetch_ms = fetch_ms;
  st_.merge_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - fetch_ms;
  st_.merge_path = "device-generic";
  return true;
}

}  // namespace uda
