// Device shuffle/merge engine implementation. See device_engine.h for the design.
#include "device_engine.h"
#include "device_ptr.h"
#include "hbm_ledger.h"
#include "merge_plan.h"
#include "sdma.h"
#include "uda/fault.h"
#include "uda/topology.h"
#include "uda/trace.h"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <stdexcept>

#include "uda/log.h"
#include "uda/vint.h"
#include "uda/thread_name.h"

namespace uda {
namespace gpu {

namespace {
constexpr int kSlots = 2;  // recv/out double buffering across rounds


double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

int64_t total_records(const std::vector<RunDesc>& runs) {
  int64_t t = 0;
  for (const auto& r : runs) t += r.nrec;
  return t;
}
}  // namespace

void hip_check(hipError_t e, const char* what, const char* file, int line) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what +
                             " at " + file + ":" + std::to_string(line));
}

// ------------------------------------------------------------------------------------ buffers
DeviceBuffer::~DeviceBuffer() { reset(); }
namespace {
// UDA_DEVICE_GUARD=1 (debug): every device buffer gets a tail of kGuardByte past its size (local
// buffers: 64 KiB more; exportable ones: their IPC padding), checked when the buffer is freed. A kernel
// writing past the end of its buffer then shows as a logged violation instead of silently changing the
// next allocation's bytes.
constexpr size_t kGuardBytes = 64 << 10;
constexpr int kGuardByte = 0xA5;
std::atomic<int64_t> g_guard_violations{0};
bool guard_enabled() {
  const char* e = std::getenv("UDA_DEVICE_GUARD");
  return e && std::atoi(e) != 0;
}
}  // namespace

int64_t device_guard_violations() { return g_guard_violations.load(); }

void DeviceBuffer::alloc_impl(size_t bytes, bool resident, bool exportable) {
  reset();
  if (bytes == 0) return;
  if (fault_hit("DEVICE_ALLOC")) throw std::runtime_error("injected device allocation failure");
  // Blocks another process may map over hipIpc (our descriptor fetch, RCCL's peer registration of
  // send/receive buffers) must stay out of the size range that hangs the importer (device_ptr.h).
  const bool guard = guard_enabled();
  const size_t held = exportable ? ipc_safe_bytes(bytes + (guard ? 1 : 0)) : bytes + (guard ? kGuardBytes : 0);
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  HbmLedger::get().on_alloc(dev, (int64_t)held, resident);
  const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
  const hipError_t e = hipMalloc(&ptr_, held);
  if (e != hipSuccess) {
    ptr_ = nullptr;
    HbmLedger::get().on_free(dev, (int64_t)held, resident);
    (void)hipGetLastError();
    const HbmLedger::Stats ls = HbmLedger::get().stats(dev);
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " allocating " +
                             std::to_string(held) + " bytes on device " + std::to_string(dev) + " (" +
                             std::to_string(free_b) + " free of " + std::to_string(total_b) +
                             "; this process: used " + std::to_string(ls.used) + ", reserved " +
                             std::to_string(ls.reserved) + ", node " + std::to_string(ls.node_bytes) +
                             ", budget " + std::to_string(ls.budget) + (HbmLedger::get().bound() ? ", in a reservation" : "") +
                             ")");
  }
  if (tt) trace::host_event("device_alloc", (int64_t)bytes, 0, tt, trace::now_ns());
  size_ = bytes;
  held_ = held;
  dev_ = dev;
  resident_ = resident;
  guarded_ = guard && held > bytes;
  if (guarded_) {  // complete before any non-blocking stream writes near it
    HIP_CHECK(hipMemsetAsync(static_cast<uint8_t*>(ptr_) + bytes, kGuardByte, std::min(held - bytes, kGuardBytes), nullptr));
    HIP_CHECK(hipStreamSynchronize(nullptr));
  }
}
void DeviceBuffer::reset() {
  if (ptr_ && guarded_) {
    const size_t n = std::min(held_ - size_, kGuardBytes);
    std::vector<uint8_t> tail(n);
    if (hipMemcpy(tail.data(), static_cast<uint8_t*>(ptr_) + size_, n, hipMemcpyDeviceToHost) == hipSuccess) {
      size_t bad = 0, first = n;
      for (size_t i = 0; i < n; ++i)
        if (tail[i] != (uint8_t)kGuardByte) {
          ++bad;
          first = std::min(first, i);
        }
      if (bad) {
        g_guard_violations.fetch_add(1);
        UDA_LOG(kError, "device buffer of %zu bytes: %zu guard bytes overwritten, the first %zu past its end", size_,
                bad, first);
      }
    }
    guarded_ = false;
  }
  if (ptr_) note_device_free(ptr_);  // an exporter's cached IPC identity of this address is stale now
  if (ptr_ && trace::host_enabled()) {
    const int64_t tt = trace::now_ns();
    (void)hipFree(ptr_);
    trace::host_event("device_free", (int64_t)size_, 0, tt, trace::now_ns());
    ptr_ = nullptr;
  }
  if (ptr_) (void)hipFree(ptr_);
  if (held_) HbmLedger::get().on_free(dev_, (int64_t)held_, resident_);
  ptr_ = nullptr;
  size_ = held_ = 0;
}

PinnedBuffer::~PinnedBuffer() { pinned_host_free(ptr_); }
PinnedPool& PinnedPool::instance() {
  static PinnedPool* pool = new PinnedPool();  // leaked on purpose: outlives every user at exit
  return *pool;
}

PinnedPool::Block PinnedPool::acquire(size_t min_bytes) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = free_.lower_bound(min_bytes);
    if (it != free_.end() && it->first <= 2 * min_bytes + PinnedArena::kBlock) {
      Block b{it->second, it->first};
      cached_ -= it->first;
      free_.erase(it);
      return b;
    }
  }
  Block b;
  // 2 MiB granules; blocks above 64 MiB in 32 MiB granules, so the next task's slightly different
  // sizes (LPQ spills, partitions) find the cached block instead of pinning a new one (tens of ms)
  const size_t gran = min_bytes > ((size_t)64 << 20) ? ((size_t)32 << 20) : ((size_t)2 << 20);
  b.size = (min_bytes + gran - 1) & ~(gran - 1);
  void* p = nullptr;
  const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
  try {
    p = pinned_host_alloc(b.size);
  } catch (const std::exception&) {
    // memory the reaper still holds, then the cache: trim and retry once
    drain_reaper();
    std::multimap<size_t, uint8_t*> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      drop.swap(free_);
      cached_ = 0;
    }
    for (auto& kv : drop) pinned_host_free(kv.second);
    try {
      p = pinned_host_alloc(b.size);
    } catch (const std::exception&) {
      throw std::runtime_error("pinned host allocation of " + std::to_string(b.size) + " bytes failed");
    }
  }
  if (tt) trace::host_event("pinned_alloc", (int64_t)b.size, (int64_t)min_bytes, tt, trace::now_ns());
  b.p = static_cast<uint8_t*>(p);
  return b;
}

void PinnedPool::release(Block b) {
  if (!b.p) return;
  std::lock_guard<std::mutex> g(mu_);
  if (cached_ + b.size > cap_) {
    // unpinning and unmapping GBs takes hundreds of ms (a 41.6 GB over-budget task spent 486 ms closing
    // on it): a reaper thread does it off the task's path
    reap_.push_back(b);
    if (!reaper_started_) {
      reaper_started_ = true;
      std::thread([this] { name_thread("uda-pin-reaper"); reaper_main(); }).detach();  // the pool is never destroyed
    }
    reap_cv_.notify_one();
    return;
  }
  free_.emplace(b.size, b.p);
  cached_ += b.size;
}

void PinnedPool::reaper_main() {
  for (;;) {
    Block b;
    {
      std::unique_lock<std::mutex> lk(mu_);
      reap_cv_.wait(lk, [&] { return !reap_.empty(); });
      b = reap_.front();
      reap_.pop_front();
      ++reaping_;
    }
    pinned_host_free(b.p);
    std::lock_guard<std::mutex> g(mu_);
    --reaping_;
    reap_cv_.notify_all();
  }
}

void PinnedPool::drain_reaper() {
  for (;;) {
    Block b;
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (reap_.empty()) {
        reap_cv_.wait(lk, [&] { return reaping_ == 0 || !reap_.empty(); });
        if (reap_.empty()) return;
      }
      b = reap_.front();
      reap_.pop_front();
    }
    pinned_host_free(b.p);
  }
}

void PinnedPool::set_cache_cap(size_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  cap_ = bytes;
}

namespace {
size_t host_memory_limit() {
  size_t lim = (size_t)sysconf(_SC_PHYS_PAGES) * (size_t)sysconf(_SC_PAGESIZE);
  if (FILE* f = std::fopen("/sys/fs/cgroup/memory.max", "r")) {  // cgroup v2 ("max" = none)
    unsigned long long v = 0;
    if (std::fscanf(f, "%llu", &v) == 1 && v > 0) lim = std::min<size_t>(lim, (size_t)v);
    std::fclose(f);
  }
  return lim;
}
}  // namespace

void PinnedPool::raise_cache_cap(size_t bytes) {
  static const size_t ceiling = host_memory_limit() / 4;
  std::lock_guard<std::mutex> g(mu_);
  cap_ = std::max(cap_, std::min(bytes, ceiling));
}

size_t PinnedPool::cached_bytes() {
  std::lock_guard<std::mutex> g(mu_);
  return cached_;
}

uint8_t* PinnedArena::alloc(size_t bytes) {
  bytes = (bytes + 255) & ~(size_t)255;
  bytes_ += bytes;
  if (bytes > kBlock / 4) {  // large request: a dedicated block, kept behind the shared one
    PinnedPool::Block b = PinnedPool::instance().acquire(std::max<size_t>(bytes, 256));
    if (last_shared_ && !blocks_.empty()) {
      blocks_.insert(blocks_.end() - 1, b);
    } else {
      blocks_.push_back(b);
      last_shared_ = false;
    }
    return b.p;
  }
  if (!last_shared_ || used_ + bytes > blocks_.back().size) {
    blocks_.push_back(PinnedPool::instance().acquire(kBlock));
    used_ = 0;
    last_shared_ = true;
  }
  uint8_t* p = blocks_.back().p + used_;
  used_ += bytes;
  return p;
}

void PinnedArena::release_all() {
  for (auto& b : blocks_) PinnedPool::instance().release(b);
  blocks_.clear();
  used_ = 0;
  last_shared_ = false;
  bytes_ = 0;
}

void PinnedBuffer::alloc(size_t bytes) {
  pinned_host_free(ptr_);
  ptr_ = nullptr;
  size_ = 0;
  if (bytes == 0) return;
  const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
  ptr_ = pinned_host_alloc(bytes);
  if (tt) trace::host_event("pinned_buf_alloc", (int64_t)bytes, -1, tt, trace::now_ns());
  size_ = bytes;
}

void PinnedBuffer::alloc_on_node(size_t bytes, int node) {
  pinned_host_free(ptr_);
  ptr_ = nullptr;
  size_ = 0;
  if (bytes == 0) return;
  const int64_t tt = trace::host_enabled() ? trace::now_ns() : 0;
  ptr_ = pinned_host_alloc(bytes, node);  // preferred-node pages, registered (sdma.h)
  if (tt) trace::host_event("pinned_buf_alloc", (int64_t)bytes, node, tt, trace::now_ns());
  size_ = bytes;
}

std::string nccl_unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

namespace {
struct StreamPool {
  std::mutex mu;
  std::map<std::pair<int, int>, std::vector<hipStream_t>> idle;  // (device, priority) -> streams
  std::map<hipStream_t, std::pair<int, int>> owner;               // every pooled stream's key
  static StreamPool& get() {
    static StreamPool* p = new StreamPool;  // never destroyed: streams outlive static teardown order
    return *p;
  }
};
}  // namespace

hipStream_t pooled_stream(int priority) {
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  StreamPool& p = StreamPool::get();
  {
    std::lock_guard<std::mutex> g(p.mu);
    auto& v = p.idle[{dev, priority}];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  std::lock_guard<std::mutex> g(p.mu);
  p.owner[s] = {dev, priority};
  return s;
}

void return_stream(hipStream_t s) {
  if (!s) return;
  StreamPool& p = StreamPool::get();
  std::lock_guard<std::mutex> g(p.mu);
  auto it = p.owner.find(s);
  if (it == p.owner.end()) {
    (void)hipStreamDestroy(s);  // not one of ours
    return;
  }
  p.idle[it->second].push_back(s);
}

void prewarm_streams(int device, int n) {
  HIP_CHECK(hipSetDevice(device));
  std::vector<hipStream_t> v;
  for (int i = 0; i < n; ++i) v.push_back(pooled_stream(0));
  for (hipStream_t s : v) return_stream(s);
}


// ------------------------------------------------------------------------------ DeviceMerger
// Per-round plan blob layout (all int64 unless noted), uploaded with one H2D copy:
//   RunDesc runs[K] | int64 elem_off[K+1] | uint8_t* bases[K] | per pass: pairs[3P], tile_prefix[P+1]
DeviceMerger::DeviceMerger(int64_t max_records, int max_runs)
    : max_records_(max_records), max_runs_(max_runs) {
  // the merge-tree buffers (2 x 16 B per record) are allocated on the tree path's first use: the
  // single-pass K-way merge, which takes every group of <= kKwMaxRuns runs, never touches them
  static const bool old_null = [] {  // tools/multirank_stress.py --old-memset 2: the r5 code here too
    const char* e = std::getenv("UDA_GEN_NULL_STREAM_MEMSET");
    return e && std::atoi(e) >= 2;
  }();
  flag_.alloc(sizeof(int));
  if (old_null) HIP_CHECK(hipMemset(flag_.as(), 0, sizeof(int)));
  else HIP_CHECK(hipMemsetAsync(flag_.as(), 0, sizeof(int), nullptr));
  int passes = 1;
  while ((1 << passes) < max_runs) ++passes;
  ++passes;  // groups that are not a power of two may need one extra copy-through level
  slot_bytes_ = (size_t)max_runs * (sizeof(RunDesc) + 2 * sizeof(int64_t) + sizeof(uint8_t*)) +
                (size_t)passes * (4 * (size_t)max_runs + 4) * sizeof(int64_t) + 64 * (size_t)(passes + 4);
  // single-pass K-way tables: runs, bases, counts, sample offsets, bound sets, group / cell tables
  slot_bytes_ += (size_t)max_runs * (sizeof(RunDesc) + 4 * sizeof(int64_t) + 2 * sizeof(int)) + 64 * 16;
  if (const char* e = std::getenv("UDA_KWAY")) kway_ = std::atoi(e) != 0;
  if (const char* e = std::getenv("UDA_KWAY_CAP")) kw_cap_ = std::atoi(e);
  if (const char* e = std::getenv("UDA_KWAY_STAGED")) kw_staged_ = std::atoi(e) != 0;
  if (kw_staged_ && kw_cap_ > 1024) kw_cap_ = 1024;  // a staged cell's records must fit LDS
  if (!kway_cap_supported(kw_cap_)) throw std::runtime_error("UDA_KWAY_CAP must be 512, 1024, 1536, 1792 or 2048");
  kw_overflow_.alloc(sizeof(int));
  if (old_null) {
    HIP_CHECK(hipMemset(kw_overflow_.as(), 0, sizeof(int)));
  } else {
    HIP_CHECK(hipMemsetAsync(kw_overflow_.as(), 0, sizeof(int), nullptr));
    // the merges run on non-blocking streams, which do not wait for the null stream
    HIP_CHECK(hipStreamSynchronize(nullptr));
  }
  slots_.resize(4);
  for (auto& s : slots_) {
    s.host.alloc(slot_bytes_);
    s.dev.alloc(slot_bytes_);
    HIP_CHECK(hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming));
  }
}

int64_t DeviceMerger::device_bytes() const {
  int64_t n = (int64_t)(elems_a_.held() + elems_b_.held() + splits_.held() + flag_.held() + kw_prof_.held() +
                        kw_overflow_.held());
  for (const auto& p : pbufs_)
    n += (int64_t)(p.samp_runs.held() + p.samp_a.held() + p.samp_b.held() + p.bounds.held() + p.split.held() +
                   p.splits.held());
  for (const auto& s : slots_) n += (int64_t)s.dev.held();
  return n;
}

DeviceMerger::~DeviceMerger() {
  for (auto& s : slots_)
    if (s.uploaded) (void)hipEventDestroy(s.uploaded);
  for (auto& p : pbufs_) {
    if (p.planned) (void)hipEventDestroy(p.planned);
    if (p.used) (void)hipEventDestroy(p.used);
  }
}

int DeviceMerger::kway_overflow_cells() {
  int v = 0;
  HIP_CHECK(hipMemcpy(&v, kw_overflow_.as(), sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

bool DeviceMerger::bad_layout() {
  int v = 0;
  HIP_CHECK(hipMemcpy(&v, flag_.as(), sizeof(int), hipMemcpyDeviceToHost));
  return v != 0;
}

int64_t DeviceMerger::merge_fixed(const std::vector<RunDesc>& runs, const std::vector<int>& group_first,
                                  uint8_t* out, hipStream_t s) {
  const int K = (int)runs.size();
  if (K > max_runs_) throw std::runtime_error("DeviceMerger: too many runs");
  if (K > 65536) throw std::runtime_error("DeviceMerger: FIXED10 mode supports <= 65536 runs");
  if (group_first.empty() || group_first.front() != 0 || group_first.back() != K)
    throw std::runtime_error("DeviceMerger: bad run groups");
  int64_t total = 0;
  for (const auto& r : runs) total += r.nrec;
  if (total > max_records_) throw std::runtime_error("DeviceMerger: round exceeds capacity");
  last_passes_ = 0;
  if (total == 0) return 0;
  if (kway_) {
    int kmax = 0;
    for (size_t g = 0; g + 1 < group_first.size(); ++g) kmax = std::max(kmax, group_first[g + 1] - group_first[g]);
    if (kmax <= kKwMaxRuns) return merge_kway(runs, group_first, out, s);
  }

  if (!elems_a_.size()) {
    elems_a_.alloc_local((size_t)std::max<int64_t>(max_records_, 1) * sizeof(Elem));
    elems_b_.alloc_local((size_t)std::max<int64_t>(max_records_, 1) * sizeof(Elem));
    // tiles per pass <= records/2048 + pairs; splits buffer sized for one pass
    const int64_t max_tiles = max_records_ / kMergeTile + max_runs_ + 2;
    splits_.alloc_local((size_t)max_tiles * sizeof(int64_t));
  }
  Slot& slot = slots_[next_slot_];
  next_slot_ = (next_slot_ + 1) % (int)slots_.size();
  if (slot.used) HIP_CHECK(hipEventSynchronize(slot.uploaded));
  slot.used = true;

  // ---- build the plan blob on the host
  uint8_t* h = slot.host.as();
  uint8_t* d = slot.dev.as();
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off = (size_t)align_up((int64_t)(off + bytes), 16);
    if (off > slot_bytes_) throw std::runtime_error("DeviceMerger: plan blob overflow");
    return o;
  };
  const size_t o_runs = carve(sizeof(RunDesc) * K);
  const size_t o_eoff = carve(sizeof(int64_t) * (K + 1));
  const size_t o_bases = carve(sizeof(uint8_t*) * K);
  std::memcpy(h + o_runs, runs.data(), sizeof(RunDesc) * K);
  int64_t* eoff = reinterpret_cast<int64_t*>(h + o_eoff);
  uint8_t** bases = reinterpret_cast<uint8_t**>(h + o_bases);
  eoff[0] = 0;
  for (int k = 0; k < K; ++k) {
    eoff[k + 1] = eoff[k] + runs[k].nrec;
    bases[k] = const_cast<uint8_t*>(runs[k].base);
  }
  const std::vector<MergePassPlan> plan = plan_merge_passes(std::vector<int64_t>(eoff, eoff + K + 1), group_first);
  std::vector<PassDesc> pds;
  for (const auto& mp : plan) {
    const size_t o_pairs = carve(sizeof(int64_t) * mp.pairs.size());
    const size_t o_tp = carve(sizeof(int64_t) * mp.tile_prefix.size());
    std::memcpy(h + o_pairs, mp.pairs.data(), sizeof(int64_t) * mp.pairs.size());
    std::memcpy(h + o_tp, mp.tile_prefix.data(), sizeof(int64_t) * mp.tile_prefix.size());
    PassDesc pd;
    pd.pairs = reinterpret_cast<const int64_t*>(d + o_pairs);
    pd.tile_prefix = reinterpret_cast<const int64_t*>(d + o_tp);
    pd.npairs = mp.npairs;
    pd.ntiles = mp.ntiles;
    pds.push_back(pd);
  }
  HIP_CHECK(hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipEventRecord(slot.uploaded, s));

  // ---- F2: keys
  Elem* cur = elems_a_.as<Elem>();
  Elem* nxt = elems_b_.as<Elem>();
  launch_extract_fixed(reinterpret_cast<const RunDesc*>(d + o_runs), reinterpret_cast<const int64_t*>(d + o_eoff), K,
                       total, cur, flag_.as<int>(), s);
  // ---- F3: merge tree (pairs never cross groups)
  for (const auto& pd : pds) {
    launch_merge_partition(cur, pd, splits_.as<int64_t>(), s);
    launch_merge_pass(cur, nxt, pd, splits_.as<int64_t>(), s);
    std::swap(cur, nxt);
  }
  last_passes_ = (int)pds.size();
  // ---- F4: gather records into merged order
  launch_gather_fixed(cur, total, reinterpret_cast<uint8_t* const*>(d + o_bases), out, s);
  return total;
}

// Tools: mean per-cell time of the k-way kernel phases (slices, F2 keys, F3 LDS merge, F4 gather)
// and the kernel span, from the per-workgroup wall-clock stamps. Synchronizes `s`.
static void report_kway_phases(const unsigned long long* dprof, int64_t ncells, hipStream_t s) {
  std::vector<unsigned long long> h((size_t)ncells * 5);
  HIP_CHECK(hipMemcpyAsync(h.data(), dprof, h.size() * 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  int dev = 0, khz = 100000;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  double sum[4] = {0, 0, 0, 0};
  unsigned long long t_min = ~0ull, t_max = 0;
  int64_t n = 0;
  for (int64_t c = 0; c < ncells; ++c) {
    const unsigned long long* p = &h[(size_t)c * 5];
    if (!p[4]) continue;  // overflow cells (PQ path) end early
    for (int k = 0; k < 4; ++k) sum[k] += (double)(p[k + 1] - p[k]);
    t_min = std::min(t_min, p[0]);
    t_max = std::max(t_max, p[4]);
    ++n;
  }
  if (!n) return;
  const double us = 1000.0 / khz;
  std::fprintf(stderr, "kway phases (mean us/cell over %lld cells): slices %.2f f2 %.2f f3 %.2f f4 %.2f | span %.1f us\n",
               (long long)n, sum[0] / n * us, sum[1] / n * us, sum[2] / n * us, sum[3] / n * us,
               (double)(t_max - t_min) * us);
}

// Single-pass K-way merge (kway.hip): sample -> merge the samples per group -> splitters ->
// per-run cell splits -> one workgroup per cell doing F2 + F3 + F4 in LDS.
int64_t DeviceMerger::merge_kway(const std::vector<RunDesc>& runs, const std::vector<int>& group_first, uint8_t* out,
                                 hipStream_t s) {
  const KwayPlan p = plan_kway(runs, group_first, s);
  return run_kway(p, out, s);
}

bool DeviceMerger::kway_applicable(const std::vector<RunDesc>& runs, const std::vector<int>& group_first) const {
  if (!kway_ || group_first.empty() || group_first.back() != (int)runs.size() || (int)runs.size() > max_runs_)
    return false;
  int64_t total = 0;
  for (const auto& r : runs) total += r.nrec;
  if (total > max_records_) return false;
  for (size_t g = 0; g + 1 < group_first.size(); ++g)
    if (group_first[g + 1] - group_first[g] > kKwMaxRuns) return false;
  return true;
}

// Cell planning of one K-way merge (sample -> merge the samples per group -> splitters -> per-run
// cell splits), enqueued on `s` into one of two plan slots. The slot's previous tiles must be done
// reading it first (device-side wait), so planning round q+1 on a side stream overlaps the tiles of
// round q on the compute stream.
DeviceMerger::KwayPlan DeviceMerger::plan_kway(const std::vector<RunDesc>& runs, const std::vector<int>& group_first,
                                               hipStream_t s) {
  const int K = (int)runs.size();
  const int G = (int)group_first.size() - 1;
  KwayPlan kp;
  kp.pslot = next_pslot_;
  next_pslot_ ^= 1;
  PlanBufs& pb = pbufs_[kp.pslot];
  if (!pb.planned) {
    HIP_CHECK(hipEventCreateWithFlags(&pb.planned, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&pb.used, hipEventDisableTiming));
  }
  if (pb.used_valid) HIP_CHECK(hipStreamWaitEvent(s, pb.used, 0));
  int kmax = 1;
  for (int g = 0; g < G; ++g) kmax = std::max(kmax, group_first[g + 1] - group_first[g]);
  const int64_t cap = kw_cap_;
  // target records per cell: cap * fill %; the rest of the capacity is the sampling slack (K * step)
  const char* fe = std::getenv("UDA_KWAY_FILL");  // read per plan: tests flip it within one process
  const int fill = fe ? std::min(90, std::max(10, std::atoi(fe))) : 65;  // profiles/r3_kway_occupancy.md
  int64_t T = cap * fill / 100;
  if (const char* e = std::getenv("UDA_KWAY_TARGET")) T = std::max<int64_t>(1, std::atoll(e));  // tests: force the PQ path
  const int64_t step = std::max<int64_t>(1, (cap - std::min<int64_t>(T, cap)) / (kmax + 2));  // cell <= T + K*step
  std::vector<int64_t> soff(K + 1, 0), nrec(K);
  std::vector<uint8_t*> bases(K);
  std::vector<int> bset(K);
  for (int g = 0; g < G; ++g)
    for (int r = group_first[g]; r < group_first[g + 1]; ++r) bset[r] = g;
  for (int r = 0; r < K; ++r) {
    nrec[r] = runs[r].nrec;
    bases[r] = const_cast<uint8_t*>(runs[r].base);
    const int64_t c = nrec[r] > step / 2 ? (nrec[r] - step / 2 + step - 1) / step : 0;
    soff[r + 1] = soff[r] + c;
  }
  const int64_t ns = soff[K];
  std::vector<int64_t> gcells(G), cell_first(G + 1, 0), gsamp(G + 1, 0), gout(G, 0);
  int64_t nbmax = 0, acc = 0;
  for (int g = 0; g < G; ++g) {
    int64_t ng = 0;
    for (int r = group_first[g]; r < group_first[g + 1]; ++r) ng += nrec[r];
    gcells[g] = std::max<int64_t>(1, (ng + T - 1) / T);
    cell_first[g + 1] = cell_first[g] + gcells[g];
    gsamp[g] = soff[group_first[g]];
    gout[g] = acc;
    acc += ng;
    nbmax = std::max(nbmax, gcells[g] - 1);
  }
  gsamp[G] = soff[K];
  const int64_t per = nbmax + 2;
  auto ensure = [](DeviceBuffer& b, size_t bytes) {
    if (b.size() < bytes) b.alloc_local(bytes + bytes / 8);
  };
  ensure(pb.samp_a, (size_t)std::max<int64_t>(ns, 1) * sizeof(Elem));
  ensure(pb.samp_b, (size_t)std::max<int64_t>(ns, 1) * sizeof(Elem));
  ensure(pb.samp_runs, (size_t)std::max<int64_t>(ns, 1) * sizeof(Elem));
  ensure(pb.bounds, (size_t)std::max<int64_t>((int64_t)G * nbmax, 1) * sizeof(Elem));
  ensure(pb.split, (size_t)K * per * sizeof(int64_t));
  ensure(pb.splits, (size_t)(ns / kMergeTile + K + 2) * sizeof(int64_t));

  Slot& slot = slots_[next_slot_];
  next_slot_ = (next_slot_ + 1) % (int)slots_.size();
  if (slot.used) HIP_CHECK(hipEventSynchronize(slot.uploaded));
  slot.used = true;
  uint8_t* h = slot.host.as();
  uint8_t* d = slot.dev.as();
  size_t off = 0;
  auto carve = [&](const void* src, size_t bytes) {
    const size_t o = off;
    off = (size_t)align_up((int64_t)(off + bytes), 16);
    if (off > slot_bytes_) throw std::runtime_error("DeviceMerger: plan blob overflow (k-way)");
    std::memcpy(h + o, src, bytes);
    return o;
  };
  const size_t o_runs = carve(runs.data(), sizeof(RunDesc) * K);
  const size_t o_bases = carve(bases.data(), sizeof(uint8_t*) * K);
  const size_t o_nrec = carve(nrec.data(), 8 * K);
  const size_t o_soff = carve(soff.data(), 8 * (K + 1));
  const size_t o_bset = carve(bset.data(), sizeof(int) * K);
  const size_t o_gf = carve(group_first.data(), sizeof(int) * (G + 1));
  const size_t o_cf = carve(cell_first.data(), 8 * (G + 1));
  const size_t o_gs = carve(gsamp.data(), 8 * (G + 1));
  const size_t o_gc = carve(gcells.data(), 8 * G);
  const size_t o_go = carve(gout.data(), 8 * G);
  std::vector<PassDesc> pds;
  for (const auto& mp : plan_merge_passes(soff, group_first)) {
    const size_t o_pairs = carve(mp.pairs.data(), 8 * mp.pairs.size());
    const size_t o_tp = carve(mp.tile_prefix.data(), 8 * mp.tile_prefix.size());
    PassDesc pd;
    pd.pairs = reinterpret_cast<const int64_t*>(d + o_pairs);
    pd.tile_prefix = reinterpret_cast<const int64_t*>(d + o_tp);
    pd.npairs = mp.npairs;
    pd.ntiles = mp.ntiles;
    pds.push_back(pd);
  }
  HIP_CHECK(hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipEventRecord(slot.uploaded, s));

  // splitters: a regular sample of every run, merged per group, every (ns_g / C_g)-th kept; the
  // per-run sample stays intact (first merge pass reads it) and brackets the split searches
  Elem* sr = pb.samp_runs.as<Elem>();
  Elem* sbuf[2] = {pb.samp_a.as<Elem>(), pb.samp_b.as<Elem>()};
  if (ns > 0)
    launch_sample_fixed(reinterpret_cast<uint8_t* const*>(d + o_bases), reinterpret_cast<const int64_t*>(d + o_nrec), K,
                        step, reinterpret_cast<const int64_t*>(d + o_soff), ns, sr, s);
  const Elem* merged = sr;
  int w = 0;
  for (const auto& pd : pds) {
    launch_merge_partition(merged, pd, pb.splits.as<int64_t>(), s);
    launch_merge_pass(merged, sbuf[w], pd, pb.splits.as<int64_t>(), s);
    merged = sbuf[w];
    w ^= 1;
  }
  launch_pick_splitters(merged, reinterpret_cast<const int64_t*>(d + o_gs), reinterpret_cast<const int64_t*>(d + o_gc),
                        G, (int)nbmax, pb.bounds.as<Elem>(), s);
  launch_split_sampled(reinterpret_cast<uint8_t* const*>(d + o_bases), reinterpret_cast<const int64_t*>(d + o_nrec), sr,
                       reinterpret_cast<const int64_t*>(d + o_soff), step,
                       nbmax > 0 ? pb.bounds.as<Elem>() : nullptr, reinterpret_cast<const int*>(d + o_bset), K,
                       (int)nbmax, pb.split.as<int64_t>(), s);
  HIP_CHECK(hipEventRecord(pb.planned, s));
  KwayDesc& kd = kp.kd;
  kd.runs = reinterpret_cast<const RunDesc*>(d + o_runs);
  kd.group_first = reinterpret_cast<const int*>(d + o_gf);
  kd.cell_first = reinterpret_cast<const int64_t*>(d + o_cf);
  kd.split = pb.split.as<int64_t>();
  kd.nbmax = (int)nbmax;
  kd.group_out = reinterpret_cast<const int64_t*>(d + o_go);
  kd.G = G;
  kd.overflow = kw_overflow_.as<int>();
  kd.bad_layout = flag_.as<int>();
  kd.cap = (int)cap;
  kd.kmax = kmax;
  // the staged kernel reads each record's words from LDS at the run's own alignment mod 16: 8-byte
  // aligned runs only (partitions of Hadoop MOF files start 2 bytes after the previous one's EOF marker)
  bool aligned8 = true;
  for (const auto& r : runs) aligned8 = aligned8 && ((uintptr_t)r.base & 7) == 0;
  kd.staged = kw_staged_ && aligned8 ? 1 : 0;
  kp.ncells = cell_first[G];
  kp.total = total_records(runs);
  return kp;
}

int64_t DeviceMerger::run_kway(const KwayPlan& kp, uint8_t* out, hipStream_t s) {
  PlanBufs& pb = pbufs_[kp.pslot];
  HIP_CHECK(hipStreamWaitEvent(s, pb.planned, 0));
  KwayDesc kd = kp.kd;
  static const bool prof = std::getenv("UDA_KWAY_PROF") != nullptr;
  if (prof) {
    auto ensure = [](DeviceBuffer& b, size_t bytes) {
      if (b.size() < bytes) b.alloc_local(bytes + bytes / 8);
    };
    ensure(kw_prof_, (size_t)kp.ncells * 5 * 8);
    HIP_CHECK(hipMemsetAsync(kw_prof_.as(), 0, (size_t)kp.ncells * 5 * 8, s));
    kd.prof = kw_prof_.as<unsigned long long>();
  }
  HIP_CHECK(hipGetLastError());  // nothing pending from the plan's launches
  launch_kway_tiles(kd, kp.ncells, out, s);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(pb.used, s));
  pb.used_valid = true;
  if (prof) report_kway_phases(kd.prof, kp.ncells, s);
  last_passes_ = 1;
  return kp.total;
}

// -------------------------------------------------------------------------------- ShuffleJob
ShuffleJob::ShuffleJob(const ShuffleConfig& cfg) : cfg_(cfg) {
  if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world)
    throw std::runtime_error("ShuffleJob: bad rank/world");
  if (cfg_.maps_per_rank < 1) throw std::runtime_error("ShuffleJob: maps_per_rank < 1");
  if (cfg_.rounds < 1) cfg_.rounds = 1;
  if (cfg_.reducers < 1) cfg_.reducers = 1;
  if (cfg_.pinned_slots < 2) cfg_.pinned_slots = 2;
  if (cfg_.d2h != "sdma" && cfg_.d2h != "hip") throw std::runtime_error("ShuffleJob: d2h must be sdma or hip");
  if (cfg_.store != "hbm" && cfg_.store != "host" && cfg_.store != "disk")
    throw std::runtime_error("unknown store tier " + cfg_.store);
  R_ = cfg_.reducers;
  Q_ = cfg_.rounds;
  C_ = R_ * Q_;
  if ((int64_t)R_ * cfg_.world * cfg_.maps_per_rank > 65536)
    throw std::runtime_error("ShuffleJob: reducers * world * maps_per_rank must be <= 65536 (merge run index)");
  HIP_CHECK(hipSetDevice(cfg_.device));
  int lo_prio = 0, hi_prio = 0;
  HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
  // HBM store: the comm stream carries RCCL and gets the high priority. Spill tiers: it carries the
  // round's H2D staging (a copy kernel reading host memory), which must not hold back the merge of
  // the previous round: the merge stream gets the high priority instead.
  const bool spill = cfg_.store != "hbm";
  HIP_CHECK(hipStreamCreateWithPriority(&s_comm_, hipStreamNonBlocking, spill ? lo_prio : hi_prio));
  HIP_CHECK(hipStreamCreateWithPriority(&s_compute_, hipStreamNonBlocking, spill ? hi_prio : lo_prio));
  HIP_CHECK(hipStreamCreateWithFlags(&s_copy_, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&s_plan_, hipStreamNonBlocking));
  buf_records_ = std::max<int64_t>(1, cfg_.kv_buf_bytes / kTeraRecordBytes);
  const int64_t buf_bytes = buf_records_ * kTeraRecordBytes;
  piece_bytes_ = std::max<int64_t>(1, cfg_.d2h_piece_bytes / buf_bytes) * buf_bytes;
  merged_ev_.resize(kSlots);
  comm_ev_.resize(kSlots);
  sent_ev_.resize(2);
  for (auto& e : merged_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : comm_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : sent_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

ShuffleJob::~ShuffleJob() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (copy_thr_.joinable()) copy_thr_.join();
  for (auto& t : consumers_)
    if (t.joinable()) t.join();
  (void)hipDeviceSynchronize();
  for (auto e : merged_ev_) (void)hipEventDestroy(e);
  if (s_stage_) (void)hipStreamDestroy(s_stage_);
  for (auto e : comm_ev_) (void)hipEventDestroy(e);
  for (auto e : sent_ev_) (void)hipEventDestroy(e);
  for (auto e : piece_ev_) (void)hipEventDestroy(e);
  if (!sdma_ && ring_) pinned_host_free(ring_);
  if (sdma_) {
    for (auto sg : piece_sig_) sdma_->destroy_signal(sg);
    sdma_->free_host(ring_);
    ring_ = nullptr;
    sdma_.reset();
  }
  exchange_.reset();
  if (s_copy_) (void)hipStreamDestroy(s_copy_);
  if (s_plan_) (void)hipStreamDestroy(s_plan_);
  if (s_comm_) (void)hipStreamDestroy(s_comm_);
  if (s_compute_) (void)hipStreamDestroy(s_compute_);
}

void ShuffleJob::init_comm(const std::string& uid) {
  if (cfg_.world == 1) return;
  HIP_CHECK(hipSetDevice(cfg_.device));
  exchange_ = make_rccl_exchange(cfg_.rank, cfg_.world, uid);
}

void ShuffleJob::init_local() {
  if (cfg_.world == 1) return;
  if (cfg_.local_group.empty()) throw std::runtime_error("init_local: config.local_group is empty");
  HIP_CHECK(hipSetDevice(cfg_.device));
  exchange_ = make_local_exchange(cfg_.local_group, cfg_.rank, cfg_.world);
}

void ShuffleJob::init_ipc(const std::string& name) {
  if (cfg_.world == 1) return;
  HIP_CHECK(hipSetDevice(cfg_.device));
  exchange_ = make_ipc_exchange(name, cfg_.rank, cfg_.world, cfg_.device);
}

std::string ShuffleJob::delivery_name() const {
  if (!cfg_.deliver_host) return "none";
  if (sdma_) return sdma_->describe() + " ring=" + ring_numa_;
  return "hip[numa=" + std::to_string(device_numa_node(cfg_.device)) + "] ring=" + ring_numa_;
}

void ShuffleJob::generate() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  const int nruns = M * W;
  run_off_.assign(nruns, 0);
  run_nrec_.assign(nruns, 0);
  mof_off_.assign(M + 1, 0);
  int64_t off = 0;
  for (int m = 0; m < M; ++m) {
    mof_off_[m] = off;
    for (int d = 0; d < W; ++d) {
      const int64_t n = cfg_.records_per_map / W + (d < cfg_.records_per_map % W ? 1 : 0);
      run_nrec_[m * W + d] = n;
      run_off_[m * W + d] = off;
      off = align_up(off + n * kTeraRecordBytes + kEofBytes, 16);
    }
    off = align_up(off, 256);
  }
  mof_off_[M] = off;
  store_bytes_ = off;
  if (disk_store()) {
    std::vector<std::string> dirs;
    for (size_t b = 0; b <= cfg_.local_dirs.size();) {
      const size_t e = cfg_.local_dirs.find(',', b);
      const std::string d = cfg_.local_dirs.substr(b, e == std::string::npos ? std::string::npos : e - b);
      if (!d.empty()) dirs.push_back(d);
      if (e == std::string::npos) break;
      b = e + 1;
    }
    disk_.reset(new DiskStore(cfg_.device, dirs, std::to_string(getpid()) + "." + std::to_string(cfg_.rank), M));
    store_base_ = store_dev_base_ = nullptr;
  } else if (host_store()) {
    hstore_.alloc((size_t)store_bytes_);
    store_base_ = hstore_.as<uint8_t>();
    void* dp = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&dp, store_base_, 0));
    store_dev_base_ = reinterpret_cast<uint8_t*>(dp);
  } else {
    store_.alloc((size_t)store_bytes_, /*resident=*/true);  // padded for hipIpc export by DeviceBuffer::alloc
    store_base_ = store_dev_base_ = store_.as<uint8_t>();
  }

  std::vector<uint8_t*> bases(nruns), gen_bases(nruns);
  std::vector<uint64_t> key_lo(nruns), key_span(nruns), seeds(nruns);
  const uint64_t step = (W == 1) ? ~0ull : (~0ull / (uint64_t)W);
  int64_t max_n = 0, max_mof = 0;
  DeviceBuffer tmp;  // host/disk tier: one MOF at a time is generated in HBM, then copied out
  if (spilled()) {
    for (int m = 0; m < M; ++m) max_mof = std::max(max_mof, mof_off_[m + 1] - mof_off_[m]);
    tmp.alloc((size_t)max_mof);
  }
  for (int m = 0; m < M; ++m)
    for (int d = 0; d < W; ++d) {
      const int r = m * W + d;
      bases[r] = disk_store() ? nullptr : store_dev_base_ + run_off_[r];
      gen_bases[r] = spilled() ? tmp.as<uint8_t>() + (run_off_[r] - mof_off_[m]) : bases[r];
      key_lo[r] = step * (uint64_t)d;
      key_span[r] = step;
      const uint64_t gmap = (uint64_t)cfg_.rank * M + m;
      seeds[r] = cfg_.seed ^ (0x9E3779B97F4A7C15ull * (gmap + 1)) ^ (0xC2B2AE3D27D4EB4Full * (d + 1));
      max_n = std::max(max_n, run_nrec_[r]);
    }
  DeviceBuffer d_b(nruns * sizeof(uint8_t*)), d_n(nruns * 8), d_lo(nruns * 8), d_sp(nruns * 8), d_sd(nruns * 8),
      d_ck(nruns * 8);
  HIP_CHECK(hipMemcpy(d_b.as(), gen_bases.data(), nruns * sizeof(uint8_t*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_n.as(), run_nrec_.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_lo.as(), key_lo.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_sp.as(), key_span.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_sd.as(), seeds.data(), nruns * 8, hipMemcpyHostToDevice));
  // on the stream the generation kernels accumulate on: a hipMemset goes to the null stream, which a
  // non-blocking stream does not wait for, and it returns before the device ran it -- the kernels then
  // added onto stale bytes or were zeroed midway, and the job's expected checksums came out wrong
  // (the r5 multi-rank "checksum mismatch" with records, order and every slice correct)
  static const bool old_memset = [] {  // tools/multirank_stress.py --old-memset: the r5 code, to show the race
    const char* e = std::getenv("UDA_GEN_NULL_STREAM_MEMSET");
    return e && std::atoi(e) != 0;
  }();
  if (old_memset)
    HIP_CHECK(hipMemset(d_ck.as(), 0, nruns * 8));
  else
    HIP_CHECK(hipMemsetAsync(d_ck.as(), 0, nruns * 8, s_compute_));
  // cfg.map_sort: the map side's own work — each partition is generated unsorted into the sort
  // workspace and the device radix sort (F8) gathers it, sorted, into the store. The checksums are
  // order-independent.
  DeviceBuffer sort_ws, d_stage;
  hipEvent_t sort_t0 = nullptr, sort_t1 = nullptr;
  struct EvGuard {
    hipEvent_t* a;
    hipEvent_t* b;
    ~EvGuard() {
      if (*a) (void)hipEventDestroy(*a);
      if (*b) (void)hipEventDestroy(*b);
    }
  } ev_guard{&sort_t0, &sort_t1};
  if (cfg_.map_sort) {
    if (max_n >= (int64_t)UINT32_MAX) throw std::runtime_error("map_sort: a run has 2^32 or more records");
    sort_ws.alloc((size_t)sort_fixed_ws_bytes(max_n));
    uint8_t* recs = sort_fixed_ws_records(sort_ws.as(), max_n);
    d_stage.alloc(sizeof(uint8_t*));
    HIP_CHECK(hipMemcpy(d_stage.as(), &recs, sizeof(uint8_t*), hipMemcpyHostToDevice));
    HIP_CHECK(hipEventCreate(&sort_t0));
    HIP_CHECK(hipEventCreate(&sort_t1));
  }
  map_sort_ms_ = 0;
  auto gen_runs = [&](int r0, int r1) {  // generate runs [r0, r1) at gen_bases
    if (!cfg_.map_sort) {
      launch_teragen(d_b.as<uint8_t*>() + r0, d_n.as<int64_t>() + r0, d_lo.as<uint64_t>() + r0,
                     d_sp.as<uint64_t>() + r0, d_sd.as<uint64_t>() + r0, r1 - r0, max_n,
                     d_ck.as<unsigned long long>() + r0, s_compute_);
      HIP_CHECK(hipGetLastError());
      return;
    }
    for (int r = r0; r < r1; ++r) {
      if (run_nrec_[r] <= 0) continue;
      launch_teragen(d_stage.as<uint8_t*>(), d_n.as<int64_t>() + r, d_lo.as<uint64_t>() + r, d_sp.as<uint64_t>() + r,
                     d_sd.as<uint64_t>() + r, 1, run_nrec_[r], d_ck.as<unsigned long long>() + r, s_compute_,
                     /*unsorted=*/1);
      HIP_CHECK(hipEventRecord(sort_t0, s_compute_));
      launch_sort_fixed_run(gen_bases[r], run_nrec_[r], sort_ws.as(), s_compute_, /*staged=*/true);
      HIP_CHECK(hipEventRecord(sort_t1, s_compute_));
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipEventSynchronize(sort_t1));  // the next run reuses the workspace's record area
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, sort_t0, sort_t1));
      map_sort_ms_ += ms;
    }
  };
  if (!spilled()) {
    gen_runs(0, nruns);
    HIP_CHECK(hipStreamSynchronize(s_compute_));
  } else {
    for (int m = 0; m < M; ++m) {
      gen_runs(m * W, (m + 1) * W);
      if (disk_store())  // map output written to its MOF file (O_DIRECT through io_uring)
        disk_->write_file(m, tmp.as<uint8_t>(), mof_off_[m + 1] - mof_off_[m], s_compute_);
      else
        HIP_CHECK(hipMemcpyAsync(store_base_ + mof_off_[m], tmp.as(), (size_t)(mof_off_[m + 1] - mof_off_[m]),
                                 hipMemcpyDeviceToHost, s_compute_));
    }
    HIP_CHECK(hipStreamSynchronize(s_compute_));
  }
  std::vector<uint64_t> ck(nruns);
  HIP_CHECK(hipMemcpy(ck.data(), d_ck.as(), nruns * 8, hipMemcpyDeviceToHost));
  dest_checksum_.assign(W, 0);
  dest_records_.assign(W, 0);
  run_gen_ck_ = ck;
  for (int m = 0; m < M; ++m)
    for (int d = 0; d < W; ++d) {
      dest_checksum_[d] += ck[m * W + d];
      dest_records_[d] += run_nrec_[m * W + d];
    }
  // persistent per-run device tables for splitting
  d_run_bases_.alloc(nruns * sizeof(uint8_t*));
  d_run_nrec_.alloc(nruns * 8);
  d_bound_set_.alloc(nruns * sizeof(int));
  std::vector<int> bset(nruns);
  for (int r = 0; r < nruns; ++r) bset[r] = r % W;
  HIP_CHECK(hipMemcpy(d_run_bases_.as(), bases.data(), nruns * sizeof(uint8_t*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_run_nrec_.as(), run_nrec_.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_bound_set_.as(), bset.data(), nruns * sizeof(int), hipMemcpyHostToDevice));
  UDA_LOG(kInfo, "rank %d generated %d MOFs, %ld bytes in %s%s", cfg_.rank, M, (long)store_bytes_,
          store_name().c_str(), cfg_.map_sort ? " (map-side device sort)" : "");
}

std::string ShuffleJob::store_name() const {
  if (disk_) return disk_->describe();
  return host_store() ? "pinned host DRAM" : "HBM";
}

void ShuffleJob::for_run_batches(
    const std::function<void(int, int, uint8_t* const*, const int64_t*, const int*)>& fn) {
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  if (!disk_store()) {
    fn(0, M * W, d_run_bases_.as<uint8_t*>(), d_run_nrec_.as<int64_t>(), d_bound_set_.as<int>());
    return;
  }
  int64_t max_mof = 0;
  for (int m = 0; m < M; ++m) max_mof = std::max(max_mof, mof_off_[m + 1] - mof_off_[m]);
  DeviceBuffer tmp((size_t)max_mof), d_b((size_t)W * sizeof(uint8_t*));
  std::vector<uint8_t*> b(W);
  for (int m = 0; m < M; ++m) {
    disk_->stage({DiskStore::Piece{m, 0, mof_off_[m + 1] - mof_off_[m], tmp.as<uint8_t>()}}, s_compute_);
    for (int d = 0; d < W; ++d) b[d] = tmp.as<uint8_t>() + (run_off_[m * W + d] - mof_off_[m]);
    HIP_CHECK(hipMemcpyAsync(d_b.as(), b.data(), (size_t)W * sizeof(uint8_t*), hipMemcpyHostToDevice, s_compute_));
    fn(m * W, W, d_b.as<uint8_t*>(), d_run_nrec_.as<int64_t>() + m * W, d_bound_set_.as<int>() + m * W);
    HIP_CHECK(hipStreamSynchronize(s_compute_));  // tmp is reused by the next MOF
  }
}

std::vector<int64_t> ShuffleJob::index_record(int m, int d) const {
  const int W = cfg_.world;
  if (m < 0 || m >= cfg_.maps_per_rank || d < 0 || d >= W) throw std::out_of_range("index_record");
  const int r = m * W + d;
  const int64_t part = run_nrec_[r] * kTeraRecordBytes + kEofBytes;
  return {run_off_[r] - mof_off_[m], part, part};
}

std::vector<uint8_t> ShuffleJob::read_partition(int m, int d) const {
  auto ir = index_record(m, d);
  if (disk_) return disk_->read_host(m, ir[0], ir[2]);
  std::vector<uint8_t> out((size_t)ir[2]);
  HIP_CHECK(hipMemcpy(out.data(), store_base_ + mof_off_[m] + ir[0], out.size(),
                      host_store() ? hipMemcpyHostToHost : hipMemcpyDeviceToHost));
  return out;
}

std::vector<std::vector<uint64_t>> ShuffleJob::sample_keys(int64_t every) {
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  const int nruns = M * W;
  every = std::max<int64_t>(1, every);
  std::vector<int64_t> soff(nruns + 1, 0);
  for (int r = 0; r < nruns; ++r) {
    const int64_t n = run_nrec_[r];
    const int64_t c = n > every / 2 ? (n - every / 2 + every - 1) / every : 0;
    soff[r + 1] = soff[r] + c;
  }
  const int64_t total = soff[nruns];
  std::vector<std::vector<uint64_t>> out(W);
  if (total == 0) return out;
  DeviceBuffer d_off((nruns + 1) * 8), d_out(total * sizeof(Elem));
  for_run_batches([&](int r0, int nr, uint8_t* const* bases, const int64_t* nrec, const int*) {
    std::vector<int64_t> rel(nr + 1);  // this batch's sample offsets, relative to its first sample
    for (int k = 0; k <= nr; ++k) rel[k] = soff[r0 + k] - soff[r0];
    if (rel[nr] == 0) return;
    HIP_CHECK(hipMemcpyAsync(d_off.as<int64_t>() + r0, rel.data(), (nr + 1) * 8, hipMemcpyHostToDevice, s_compute_));
    launch_sample_fixed(bases, nrec, nr, every, d_off.as<int64_t>() + r0, rel[nr], d_out.as<Elem>() + soff[r0],
                        s_compute_);
    HIP_CHECK(hipStreamSynchronize(s_compute_));  // rel is reused
  });
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  std::vector<Elem> h(total);
  HIP_CHECK(hipMemcpy(h.data(), d_out.as(), total * sizeof(Elem), hipMemcpyDeviceToHost));
  for (int r = 0; r < nruns; ++r) {
    auto& v = out[r % W];
    for (int64_t i = soff[r]; i < soff[r + 1]; ++i) {
      v.push_back(h[i].hi);
      v.push_back(h[i].lo);
    }
  }
  return out;
}

void ShuffleJob::set_bounds(const std::vector<uint64_t>& bounds) {
  const int W = cfg_.world;
  if ((int64_t)bounds.size() != (int64_t)W * (C_ - 1) * 2)
    throw std::runtime_error("set_bounds: expected world*(reducers*rounds-1)*2 values");
  bounds_ = bounds;
  if (C_ > 1) {
    d_bounds_.alloc(bounds.size() * 8);
    HIP_CHECK(hipMemcpy(d_bounds_.as(), bounds.data(), bounds.size() * 8, hipMemcpyHostToDevice));
  }
}

// Round volumes, once per job: the cell split of every local run, the counts exchange (every
// reducer learns what each peer will send it in each round) and, for world > 1, the checksum of
// every slice a peer will send (exchange verification in validated steps).
void ShuffleJob::compute_plans() {
  const int M = cfg_.maps_per_rank, W = cfg_.world, me = cfg_.rank;
  const int nruns = M * W;
  if (C_ > 1 && bounds_.empty()) throw std::runtime_error("reducers*rounds > 1 requires set_bounds()");
  const int64_t per = C_ + 1;
  d_split_out_.alloc((size_t)nruns * per * 8);
  for_run_batches([&](int r0, int nr, uint8_t* const* bases, const int64_t* nrec, const int* bset) {
    launch_split_fixed(bases, nrec, C_ > 1 ? d_bounds_.as<Elem>() : nullptr, bset, nr, C_ - 1,
                       d_split_out_.as<int64_t>() + (size_t)r0 * per, s_compute_);
  });
  split_pos_.assign((size_t)nruns * per, 0);
  HIP_CHECK(hipMemcpyAsync(split_pos_.data(), d_split_out_.as(), split_pos_.size() * 8, hipMemcpyDeviceToHost,
                           s_compute_));
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  auto pos = [&](int r, int c) { return split_pos_[(size_t)r * per + c]; };
  const size_t n_per_peer = (size_t)Q_ * R_ * M;  // counts per (peer): [q][i][m]
  std::vector<int64_t> send_counts((size_t)W * n_per_peer), recv_counts((size_t)W * n_per_peer);
  for (int p = 0; p < W; ++p)
    for (int q = 0; q < Q_; ++q)
      for (int i = 0; i < R_; ++i)
        for (int m = 0; m < M; ++m) {
          const int r = m * W + p, c = i * Q_ + q;
          send_counts[(size_t)p * n_per_peer + ((size_t)q * R_ + i) * M + m] = pos(r, c + 1) - pos(r, c);
        }
  // checksums of every (run, cell) slice of the local runs: what this rank sends (exchange
  // verification at the peers) and its own cells (checked where the merge reads them); then laid out
  // [p][q][i][m] like the counts
  std::vector<int64_t> cell_ck((size_t)nruns * C_, 0);
  {
    DeviceBuffer d_sl((size_t)nruns * C_ * sizeof(RunDesc)), d_ck((size_t)nruns * C_ * 8);
    for_run_batches([&](int r0, int nr, uint8_t* const* bases, const int64_t*, const int*) {
      std::vector<uint8_t*> hb(nr);
      HIP_CHECK(hipMemcpyAsync(hb.data(), bases, (size_t)nr * sizeof(uint8_t*), hipMemcpyDeviceToHost, s_compute_));
      HIP_CHECK(hipStreamSynchronize(s_compute_));
      std::vector<RunDesc> sl((size_t)nr * C_);
      int64_t max_n = 0;
      for (int k = 0; k < nr; ++k)
        for (int c = 0; c < C_; ++c) {
          RunDesc& d = sl[(size_t)k * C_ + c];
          d.base = hb[k] + pos(r0 + k, c) * kTeraRecordBytes;
          d.nrec = pos(r0 + k, c + 1) - pos(r0 + k, c);
          d.nbytes = d.nrec * kTeraRecordBytes;
          d.offsets = nullptr;
          max_n = std::max(max_n, d.nrec);
        }
      HIP_CHECK(hipMemcpyAsync(d_sl.as(), sl.data(), sl.size() * sizeof(RunDesc), hipMemcpyHostToDevice, s_compute_));
      for (size_t b = 0; b < sl.size(); b += 65535) {
        const int n = (int)std::min<size_t>(65535, sl.size() - b);
        launch_slice_checksums(d_sl.as<RunDesc>() + b, n, max_n, d_ck.as<unsigned long long>() + b, s_compute_);
      }
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(cell_ck.data() + (size_t)r0 * C_, d_ck.as(), sl.size() * 8, hipMemcpyDeviceToHost,
                               s_compute_));
      HIP_CHECK(hipStreamSynchronize(s_compute_));
    });
  }
  std::vector<int64_t> send_ck((size_t)W * n_per_peer), recv_ck((size_t)W * n_per_peer, 0);
  for (int p = 0; p < W; ++p)
    for (int q = 0; q < Q_; ++q)
      for (int i = 0; i < R_; ++i)
        for (int m = 0; m < M; ++m)
          send_ck[(size_t)p * n_per_peer + ((size_t)q * R_ + i) * M + m] = cell_ck[(size_t)(m * W + p) * C_ + i * Q_ + q];
  if (W == 1) {
    recv_counts = send_counts;
    recv_ck = send_ck;
  } else {
    if (!exchange_) throw std::runtime_error("world > 1 requires init_comm() or init_local()");
    exchange_->alltoall_i64(send_counts.data(), recv_counts.data(), n_per_peer, s_comm_);
    exchange_->alltoall_i64(send_ck.data(), recv_ck.data(), n_per_peer, s_comm_);
  }
  // The generation-time checksum of every run (what a validated step is checked against) must be what
  // the store holds: a mismatch is a wrong expectation, not a shuffle error. Checked after the
  // collectives, so a failing rank never leaves its peers waiting in one.
  for (int r = 0; r < nruns && (size_t)r < run_gen_ck_.size(); ++r) {
    uint64_t sum = 0;
    for (int c = 0; c < C_; ++c) sum += (uint64_t)cell_ck[(size_t)r * C_ + c];
    if (sum != run_gen_ck_[(size_t)r])
      throw std::runtime_error("plan: map output run " + std::to_string(r) + " of rank " + std::to_string(me) +
                               " holds records whose checksum differs from the one its generation computed");
  }
  // own cells: this rank's plan-time checksums, whatever the counts exchange carried for the self entry
  for (int q = 0; q < Q_; ++q)
    for (int i = 0; i < R_; ++i)
      for (int m = 0; m < M; ++m)
        recv_ck[(size_t)me * n_per_peer + ((size_t)q * R_ + i) * M + m] =
            send_ck[(size_t)me * n_per_peer + ((size_t)q * R_ + i) * M + m];
  expect_group_ck_.assign((size_t)Q_ * R_, 0);
  for (int q = 0; q < Q_; ++q)
    for (int s = 0; s < W; ++s)
      for (int i = 0; i < R_; ++i)
        for (int m = 0; m < M; ++m)
          expect_group_ck_[(size_t)q * R_ + i] += (uint64_t)recv_ck[(size_t)s * n_per_peer + ((size_t)q * R_ + i) * M + m];

  plans_.assign(Q_, RoundPlan());
  reducer_records_.assign(R_, 0);
  max_round_records_ = 0;
  int64_t max_slot_bytes = 0, max_send = 0;
  verify_n_.assign(Q_, 0);
  verify_max_nrec_.assign(Q_, 0);
  std::vector<std::vector<RunDesc>> vruns(Q_);
  std::vector<std::vector<int64_t>> vexp(Q_);
  for (int q = 0; q < Q_; ++q) {
    RoundPlan& rp = plans_[q];
    rp.send.assign(W, {});
    rp.self_beg.assign((size_t)R_ * M, 0);
    for (int i = 0; i < R_; ++i)
      for (int m = 0; m < M; ++m) rp.self_beg[(size_t)i * M + m] = pos(m * W + me, i * Q_ + q);
    for (int k = 1; k < W; ++k) {
      const int p = (me + k) % W;
      for (int i = 0; i < R_; ++i)
        for (int m = 0; m < M; ++m) {
          const int r = m * W + p, c = i * Q_ + q;
          const int64_t cnt = pos(r, c + 1) - pos(r, c);
          if (cnt <= 0) continue;
          // disk store: the span holds the file offset (staged at run time, see run_step)
          rp.send[p].push_back(Span{store_base_ + run_off_[r] + pos(r, c) * kTeraRecordBytes, cnt * kTeraRecordBytes});
          rp.send_bytes += cnt * kTeraRecordBytes;
        }
    }
    max_send = std::max(max_send, rp.send_bytes);
    rp.recv_cnt.assign((size_t)W * R_ * M, 0);
    rp.recv_off.assign((size_t)W * R_ * M, -1);
    rp.group_recs.assign(R_, 0);
    int64_t off = 0;
    for (int s = 0; s < W; ++s)
      for (int i = 0; i < R_; ++i)
        for (int j = 0; j < M; ++j) {
          const size_t x = ((size_t)s * R_ + i) * M + j;
          const int64_t cnt = recv_counts[(size_t)s * n_per_peer + ((size_t)q * R_ + i) * M + j];
          rp.recv_cnt[x] = cnt;
          rp.group_recs[i] += cnt;
          if (s == me && !spilled()) continue;  // read in place from the HBM store
          rp.recv_off[x] = off;
          off += cnt * kTeraRecordBytes;
        }
    max_slot_bytes = std::max(max_slot_bytes, off);
    for (int i = 0; i < R_; ++i) {
      rp.recv_records += rp.group_recs[i];
      reducer_records_[i] += rp.group_recs[i];
    }
    max_round_records_ = std::max(max_round_records_, rp.recv_records);
    if (W > 1) {
      for (int s = 0; s < W; ++s) {
        if (s == me) continue;
        for (int i = 0; i < R_; ++i)
          for (int j = 0; j < M; ++j) {
            const size_t x = ((size_t)s * R_ + i) * M + j;
            if (rp.recv_cnt[x] <= 0) continue;
            RunDesc d;
            d.base = nullptr;  // filled in once the receive slots exist
            d.nrec = rp.recv_cnt[x];
            d.nbytes = rp.recv_off[x];  // temporarily: offset in the slot
            d.offsets = nullptr;
            vruns[q].push_back(d);
            vexp[q].push_back(recv_ck[(size_t)s * n_per_peer + ((size_t)q * R_ + i) * M + j]);
            verify_max_nrec_[q] = std::max(verify_max_nrec_[q], d.nrec);
          }
      }
      verify_n_[q] = (int)vruns[q].size();
    }
  }

  // ---- buffers
  merger_.reset(new DeviceMerger(max_round_records_, R_ * W * M));
  const size_t out_bytes = (size_t)std::max<int64_t>(1, max_round_records_) * kTeraRecordBytes;
  out_slots_.clear();
  out_slots_.resize(kSlots);
  for (auto& b : out_slots_) b.alloc(out_bytes);
  recv_slots_.clear();
  if (staged()) {
    recv_slots_.resize(kSlots);
    for (auto& b : recv_slots_) b.alloc((size_t)std::max<int64_t>(max_slot_bytes, 16));
  }
  // spill tiers at world > 1: peers never read the host store (device memory only, for every
  // exchange backend); the round's outgoing slices are staged into HBM, double-buffered so the
  // staging of round q+1 overlaps the exchange of round q
  for (auto& b : send_staging_) b.reset();
  if (W > 1 && spilled())
    for (auto& b : send_staging_) b.alloc((size_t)std::max<int64_t>(max_send, 16));
  if (W > 1) exchange_->reserve(max_send);
  for (int q = 0; q < Q_; ++q) {
    RoundPlan& rp = plans_[q];
    rp.staged_send.assign(W, {});
    rp.staged_recv.assign(W, {});
    if (W == 1 || !spilled()) continue;
    int64_t off = 0;
    for (int p = 0; p < W; ++p) {
      const int64_t beg = off;
      for (const Span& sp : rp.send[p]) off += sp.bytes;
      if (off > beg) rp.staged_send[p].push_back(Span{send_staging_[q & 1].as<uint8_t>() + beg, off - beg});
    }
    uint8_t* rbuf = recv_slots_[q % kSlots].as<uint8_t>();
    for (int s = 0; s < W; ++s) {
      if (s == me) continue;
      int64_t first = -1, total = 0;
      for (int i = 0; i < R_; ++i)
        for (int j = 0; j < M; ++j) {
          const size_t x = ((size_t)s * R_ + i) * M + j;
          const int64_t b = rp.recv_cnt[x] * kTeraRecordBytes;
          if (b <= 0) continue;
          if (first < 0) first = rp.recv_off[x];
          if (rp.recv_off[x] != first + total) throw std::runtime_error("plan: a source's slices are not contiguous");
          total += b;
        }
      if (total > 0) rp.staged_recv[s].push_back(Span{rbuf + first, total});
    }
  }
  d_validate_.alloc(64 + (size_t)2 * R_ * sizeof(Elem));
  // exchange verification tables
  d_verify_runs_.clear();
  d_verify_expect_.clear();
  d_verify_runs_.resize(Q_);
  d_verify_expect_.resize(Q_);
  int max_v = 0;
  for (int q = 0; q < Q_; ++q) {
    if (verify_n_[q] == 0) continue;
    for (auto& d : vruns[q]) {
      d.base = recv_slots_[q % kSlots].as<uint8_t>() + d.nbytes;
      d.nbytes = d.nrec * kTeraRecordBytes;
    }
    d_verify_runs_[q].alloc(vruns[q].size() * sizeof(RunDesc));
    d_verify_expect_[q].alloc(vexp[q].size() * 8);
    HIP_CHECK(hipMemcpy(d_verify_runs_[q].as(), vruns[q].data(), vruns[q].size() * sizeof(RunDesc),
                        hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_verify_expect_[q].as(), vexp[q].data(), vexp[q].size() * 8, hipMemcpyHostToDevice));
    max_v = std::max(max_v, verify_n_[q]);
  }
  // own cells, where the merge reads them (build_runs in run_step)
  d_own_runs_.clear();
  d_own_expect_.clear();
  d_own_runs_.resize(Q_);
  d_own_expect_.resize(Q_);
  own_n_.assign(Q_, 0);
  own_max_nrec_.assign(Q_, 0);
  for (int q = 0; q < Q_; ++q) {
    const RoundPlan& rp = plans_[q];
    std::vector<RunDesc> v;
    std::vector<int64_t> e;
    for (int i = 0; i < R_; ++i)
      for (int j = 0; j < M; ++j) {
        const size_t x = ((size_t)me * R_ + i) * M + j;
        if (rp.recv_cnt[x] <= 0) continue;
        RunDesc d;
        d.nrec = rp.recv_cnt[x];
        d.nbytes = d.nrec * kTeraRecordBytes;
        d.offsets = nullptr;
        d.base = rp.recv_off[x] >= 0 ? recv_slots_[q % kSlots].as<uint8_t>() + rp.recv_off[x]
                                     : store_dev_base_ + run_off_[j * W + me] + rp.self_beg[(size_t)i * M + j] * kTeraRecordBytes;
        v.push_back(d);
        e.push_back(cell_ck[(size_t)(j * W + me) * C_ + i * Q_ + q]);
        own_max_nrec_[q] = std::max(own_max_nrec_[q], d.nrec);
      }
    own_n_[q] = (int)v.size();
    max_v = std::max(max_v, own_n_[q]);
    if (v.empty()) continue;
    d_own_runs_[q].alloc(v.size() * sizeof(RunDesc));
    d_own_expect_[q].alloc(e.size() * 8);
    HIP_CHECK(hipMemcpy(d_own_runs_[q].as(), v.data(), v.size() * sizeof(RunDesc), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_own_expect_[q].as(), e.data(), e.size() * 8, hipMemcpyHostToDevice));
  }
  if (max_v > 65535) throw std::runtime_error("exchange verification: too many slices per round");
  if (max_v > 0) d_verify_got_.alloc((size_t)max_v * 8);
  d_diag_.alloc((size_t)Q_ * diag_stride() * 8);
  d_d2h_runs_.alloc((size_t)R_ * sizeof(RunDesc));
  d_d2h_ck_.alloc((size_t)R_ * 8);
  // pinned-DRAM tier: each round's H2D (own cells into the receive slot, and for W > 1 the outgoing
  // slices into the send staging) is one batched-copy launch over fixed descriptors. The kernel reads
  // the pinned store over PCIe; hipMemcpyAsync would queue these copies on the same SDMA engine as
  // the D2H delivery and serialize the two directions of the link.
  h2d_descs_.clear();
  if (const char* e = std::getenv("UDA_H2D_BLOCKS")) h2d_blocks_ = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("UDA_H2D_SDMA")) sdma_h2d_ = std::atoi(e) != 0;
  h2d_n_.assign(Q_, 0);
  h2d_max_.assign(Q_, 0);
  if (host_store()) {
    const int me = cfg_.rank;
    h2d_descs_.resize(Q_);
    for (int q = 0; q < Q_; ++q) {
      const RoundPlan& rp = plans_[q];
      uint8_t* rbuf = recv_slots_[q % kSlots].as<uint8_t>();
      std::vector<CopyDesc> v;
      for (int i = 0; i < R_; ++i)
        for (int j = 0; j < M; ++j) {
          const size_t x = ((size_t)me * R_ + i) * M + j;
          const int64_t cnt = rp.recv_cnt[x];
          if (cnt <= 0) continue;
          const int64_t at = run_off_[j * W + me] + rp.self_beg[(size_t)i * M + j] * kTeraRecordBytes;
          v.push_back(CopyDesc{store_dev_base_ + at, rbuf + rp.recv_off[x], cnt * kTeraRecordBytes});
        }
      if (W > 1) {  // outgoing slices into the round's send staging (same layout as staged_send)
        int64_t off = 0;
        for (int p2 = 0; p2 < W; ++p2)
          for (const Span& sp : rp.send[p2]) {
            v.push_back(CopyDesc{store_dev_base_ + (sp.ptr - store_base_), send_staging_[q & 1].as<uint8_t>() + off,
                                 sp.bytes});
            off += sp.bytes;
          }
      }
      for (const CopyDesc& d : v) h2d_max_[q] = std::max(h2d_max_[q], d.bytes);
      h2d_n_[q] = (int)v.size();
      if (v.empty()) continue;
      h2d_descs_[q].alloc(v.size() * sizeof(CopyDesc));
      HIP_CHECK(hipMemcpy(h2d_descs_[q].as(), v.data(), v.size() * sizeof(CopyDesc), hipMemcpyHostToDevice));
    }
  }
}

void ShuffleJob::plan() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  compute_plans();
  if (cfg_.deliver_host && !copy_thr_.joinable()) {
    const size_t ring_bytes = (size_t)piece_bytes_ * cfg_.pinned_slots;
    if (cfg_.d2h == "sdma") {
      sdma_.reset(new SdmaEngine(cfg_.device));
      ring_ = static_cast<uint8_t*>(sdma_->alloc_host(ring_bytes));
      piece_sig_.resize(cfg_.pinned_slots);
      for (auto& sg : piece_sig_) sg = sdma_->make_signal();
    } else {
      ring_ = static_cast<uint8_t*>(hip_host_alloc_on_node(ring_bytes, device_numa_node(cfg_.device)));
      piece_ev_.resize(cfg_.pinned_slots);
      for (auto& e : piece_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // first touch from this thread: the pages land where the allocation policy put them
    for (size_t o = 0; o < ring_bytes; o += 4096) ring_[o] = 0;
    ring_numa_ = numa_residency(ring_);
    pinned_free_.assign(cfg_.pinned_slots, true);
    items_.assign(R_, {});
    eof_bufs_.clear();
    for (int i = 0; i < R_; ++i) eof_bufs_.emplace_back(new uint8_t[(size_t)cfg_.kv_buf_bytes + 16]);
    copy_thr_ = std::thread([this] { name_thread("uda-copy"); copy_loop(); });
    for (int i = 0; i < R_; ++i) consumers_.emplace_back([this, i] { name_thread("uda-consume"); consume_loop(i); });
  }
  UDA_LOG(kInfo, "rank %d planned %d reducers x %d rounds, max round %ld records, delivery %s", cfg_.rank, R_, Q_,
          (long)max_round_records_, delivery_name().c_str());
}

void ShuffleJob::wait_exchange_ok() {
  if (exchange_) exchange_->check();
}

// Copy thread: merged rounds -> D2H pieces in the pinned ring, per reducer, in round order.
void ShuffleJob::copy_loop() {
  try {
    bind_thread_to_cpus(device_consumer_cpus(cfg_.device));
    HIP_CHECK(hipSetDevice(cfg_.device));
    for (;;) {
      RoundOut r;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !round_q_.empty(); });
        if (stop_) return;
        r = std::move(round_q_.front());
        round_q_.pop_front();
      }
      HIP_CHECK(hipEventSynchronize(merged_ev_[r.slot]));
      const uint8_t* src = out_slots_[r.slot].as<uint8_t>();
      const bool last_round = (r.q == Q_ - 1);
      bool check;
      {
        std::lock_guard<std::mutex> g(mu_);
        check = step_check_delivery_;
      }
      if (check) {  // the output slot as the D2H is about to read it, per reducer
        std::vector<RunDesc> gr(R_);
        int64_t o = 0, mx = 0;
        for (int i = 0; i < R_; ++i) {
          gr[i].base = src + o * kTeraRecordBytes;
          gr[i].nrec = r.group_recs[i];
          gr[i].nbytes = gr[i].nrec * kTeraRecordBytes;
          gr[i].offsets = nullptr;
          o += r.group_recs[i];
          mx = std::max(mx, r.group_recs[i]);
        }
        std::vector<uint64_t> ck(R_, 0);
        HIP_CHECK(hipMemcpyAsync(d_d2h_runs_.as(), gr.data(), (size_t)R_ * sizeof(RunDesc), hipMemcpyHostToDevice, s_copy_));
        launch_slice_checksums(d_d2h_runs_.as<RunDesc>(), R_, std::max<int64_t>(mx, 1),
                               d_d2h_ck_.as<unsigned long long>(), s_copy_);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(ck.data(), d_d2h_ck_.as(), (size_t)R_ * 8, hipMemcpyDeviceToHost, s_copy_));
        HIP_CHECK(hipStreamSynchronize(s_copy_));
        std::lock_guard<std::mutex> g(mu_);
        for (int i = 0; i < R_; ++i) pre_d2h_ck_[(size_t)r.q * R_ + i] = ck[i];
      }
      std::vector<int> used;
      int64_t goff = 0;
      for (int i = 0; i < R_; ++i) {
        const int64_t bytes = r.group_recs[i] * kTeraRecordBytes;
        if (bytes == 0 && last_round) {
          {
            std::lock_guard<std::mutex> g(mu_);
            items_[i].push_back(Item{-1, 0, true, now_ms(), r.q});
          }
          cv_.notify_all();
        }
        for (int64_t off = 0; off < bytes;) {
          const int64_t len = std::min(piece_bytes_, bytes - off);
          int k = -1;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] {
              if (stop_) return true;
              for (bool f : pinned_free_)
                if (f) return true;
              return false;
            });
            if (stop_) return;
            for (int x = 0; x < (int)pinned_free_.size(); ++x)
              if (pinned_free_[x]) {
                k = x;
                break;
              }
            pinned_free_[k] = false;
          }
          uint8_t* dst = ring_ + (int64_t)k * piece_bytes_;
          const uint8_t* from = src + goff + off;
          if (sdma_) {
            SdmaEngine::arm(piece_sig_[k], sdma_->parts((size_t)len, cfg_.d2h_engines));
            sdma_->copy_d2h(dst, from, (size_t)len, piece_sig_[k], cfg_.d2h_engines);
          } else {
            HIP_CHECK(hipMemcpyAsync(dst, from, (size_t)len, hipMemcpyDeviceToHost, s_copy_));
            HIP_CHECK(hipEventRecord(piece_ev_[k], s_copy_));
          }
          off += len;
          used.push_back(k);
          {
            std::lock_guard<std::mutex> g(mu_);
            items_[i].push_back(Item{k, len, last_round && off >= bytes, now_ms(), r.q});
          }
          cv_.notify_all();
        }
        goff += bytes;
      }
      // the output slot is free once every piece of this round has landed in the ring
      for (int k : used) {
        if (sdma_)
          SdmaEngine::wait(piece_sig_[k]);
        else
          HIP_CHECK(hipEventSynchronize(piece_ev_[k]));
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        out_free_[r.q] = 1;
      }
      cv_.notify_all();
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> g(mu_);
    if (step_error_msg_.empty()) step_error_msg_ = std::string("delivery copy thread: ") + e.what();
    stop_ = true;
    cv_.notify_all();
  }
}

// Consumer thread of reducer i: the "Java side" hand-off. Buffers hold whole records and are at
// most kv_buf_bytes; the reducer's final buffer carries the IFile EOF marker (-1, -1).
void ShuffleJob::consume_loop(int i) {
  try {
    bind_thread_to_cpus(device_consumer_cpus(cfg_.device));
    HIP_CHECK(hipSetDevice(cfg_.device));
    const int64_t buf_bytes = buf_records_ * kTeraRecordBytes;
    uint8_t* eb = eof_bufs_[i].get();
    for (;;) {
      Item it;
      bool check;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !items_[i].empty(); });
        if (stop_) return;
        it = items_[i].front();
        items_[i].pop_front();
        check = step_check_delivery_;
      }
      uint64_t got_ck = 0;
      int err = 0;
      int64_t nb = 0;
      double waited = 0;
      bool eof_sent = false;
      if (it.pslot >= 0) {
        if (sdma_)
          SdmaEngine::wait(piece_sig_[it.pslot]);
        else
          HIP_CHECK(hipEventSynchronize(piece_ev_[it.pslot]));
        waited = now_ms() - it.issued_ms;
        const uint8_t* base = ring_ + (int64_t)it.pslot * piece_bytes_;
        if (check)
          for (int64_t off = 0; off + kTeraRecordBytes <= it.bytes; off += kTeraRecordBytes)
            got_ck += record_hash(base + off, kTeraRecordBytes);
        for (int64_t off = 0; off < it.bytes; off += buf_bytes) {
          const int64_t len = std::min(buf_bytes, it.bytes - off);
          const bool final_chunk = it.last && off + len >= it.bytes;
          if (final_chunk && len + kEofBytes <= cfg_.kv_buf_bytes) {
            std::memcpy(eb, base + off, (size_t)len);
            eb[len] = 0xFF;
            eb[len + 1] = 0xFF;
            if (sink_ && !err) err = sink_(i, eb, len + kEofBytes);
            eof_sent = true;
          } else if (sink_ && !err) {
            err = sink_(i, base + off, len);
          }
          ++nb;
        }
      }
      if (it.last && !eof_sent) {  // EOF did not fit (or no final data): a separate buffer
        eb[0] = 0xFF;
        eb[1] = 0xFF;
        if (sink_ && !err) err = sink_(i, eb, kEofBytes);
        ++nb;
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        if (it.pslot >= 0) pinned_free_[it.pslot] = true;
        if (check && it.q >= 0 && it.q < Q_) delivered_ck_[(size_t)it.q * R_ + i] += got_ck;
        step_buffers_ += nb;
        step_d2h_ms_ += waited;
        if (err && !step_error_) step_error_ = err;
        if (it.last) ++eof_count_;
      }
      cv_.notify_all();
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> g(mu_);
    if (step_error_msg_.empty()) step_error_msg_ = std::string("delivery consumer thread: ") + e.what();
    stop_ = true;
    cv_.notify_all();
  }
}

void ShuffleJob::refresh_plan() {
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  const int nruns = M * W;
  const int64_t per = C_ + 1;
  for_run_batches([&](int r0, int nr, uint8_t* const* bases, const int64_t* nrec, const int* bset) {
    launch_split_fixed(bases, nrec, C_ > 1 ? d_bounds_.as<Elem>() : nullptr, bset, nr, C_ - 1,
                       d_split_out_.as<int64_t>() + (size_t)r0 * per, s_compute_);
  });
  std::vector<int64_t> pos((size_t)nruns * per);
  HIP_CHECK(hipMemcpyAsync(pos.data(), d_split_out_.as(), pos.size() * 8, hipMemcpyDeviceToHost, s_compute_));
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  if (pos != split_pos_) throw std::runtime_error("replan: the map outputs changed since plan()");
  if (W == 1) return;
  const size_t n_per_peer = (size_t)Q_ * R_ * M;
  std::vector<int64_t> send((size_t)W * n_per_peer), recv((size_t)W * n_per_peer);
  for (int p = 0; p < W; ++p)
    for (int q = 0; q < Q_; ++q)
      for (int i = 0; i < R_; ++i)
        for (int m = 0; m < M; ++m) {
          const int r = m * W + p, c = i * Q_ + q;
          send[(size_t)p * n_per_peer + ((size_t)q * R_ + i) * M + m] = pos[(size_t)r * per + c + 1] - pos[(size_t)r * per + c];
        }
  exchange_->alltoall_i64(send.data(), recv.data(), n_per_peer, s_comm_);
  for (int q = 0; q < Q_; ++q)
    for (int s = 0; s < W; ++s)
      for (int i = 0; i < R_; ++i)
        for (int j = 0; j < M; ++j)
          if (recv[(size_t)s * n_per_peer + ((size_t)q * R_ + i) * M + j] !=
              plans_[q].recv_cnt[((size_t)s * R_ + i) * M + j])
            throw std::runtime_error("replan: a peer's counts changed since plan()");
}

// Validate steps: where a wrong total checksum came from. Per (round q, reducer i): the received
// slices and own cells against their plan-time checksums right before and right after the merge, the
// merged output against the sum of its inputs, and (check_delivery) the output slot right before its
// D2H and the bytes the consumer received against the merged output.
void ShuffleJob::localize_mismatch(StepStats& st) {
  const int F = diag_stride();
  std::vector<uint64_t> dg((size_t)Q_ * F);
  HIP_CHECK(hipMemcpy(dg.data(), d_diag_.as(), dg.size() * 8, hipMemcpyDeviceToHost));
  std::vector<uint64_t> pre_d2h, deliv;
  bool check;
  {
    std::lock_guard<std::mutex> g(mu_);
    pre_d2h = pre_d2h_ck_;
    deliv = delivered_ck_;
    check = step_check_delivery_;
  }
  st.pre_merge_errors = st.own_errors = st.merge_errors = 0;
  st.pre_d2h_errors = st.delivery_errors = check ? 0 : -1;
  std::string first[5];
  auto note = [](std::string& f, const char* what, int q, int i, uint64_t a, uint64_t b) {
    if (!f.empty()) return;
    char buf[160];
    std::snprintf(buf, sizeof(buf), "%s: round %d reducer %d (%016llx vs %016llx)", what, q, i, (unsigned long long)a,
                  (unsigned long long)b);
    f = buf;
  };
  for (int q = 0; q < Q_; ++q) {
    const uint64_t* d = &dg[(size_t)q * F];
    st.pre_merge_errors += (int64_t)d[0];
    st.own_errors += (int64_t)(d[2] + d[3]);
    if (d[0]) note(first[0], "received slices wrong before the merge", q, -1, d[0], d[1]);
    if (d[2] || d[3]) note(first[1], "own cells wrong (before, after the merge)", q, -1, d[2], d[3]);
    for (int i = 0; i < R_; ++i) {
      const uint64_t merged = d[4 + i], expect = expect_group_ck_[(size_t)q * R_ + i];
      if (merged != expect) {
        ++st.merge_errors;
        note(first[2], "merged output differs from its inputs", q, i, merged, expect);
      }
      if (!check) continue;
      if (pre_d2h[(size_t)q * R_ + i] != merged) {
        ++st.pre_d2h_errors;
        note(first[3], "output slot changed between the merge and its D2H", q, i, pre_d2h[(size_t)q * R_ + i], merged);
      }
      if (deliv[(size_t)q * R_ + i] != merged) {
        ++st.delivery_errors;
        note(first[4], "consumer received other bytes than the merge wrote", q, i, deliv[(size_t)q * R_ + i], merged);
      }
    }
  }
  st.diag.clear();
  for (const auto& f : first)
    if (!f.empty()) st.diag += (st.diag.empty() ? "" : "; ") + f;
}

StepStats ShuffleJob::run_step(bool validate) {
  trace::Range tr_step("uda.step");
  HIP_CHECK(hipSetDevice(cfg_.device));
  if (!merger_) throw std::runtime_error("run_step before plan()");
  StepStats st;
  st.validated = validate;
  const double t0 = now_ms();
  const int M = cfg_.maps_per_rank, W = cfg_.world, me = cfg_.rank;
  const bool deliver = cfg_.deliver_host;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) throw std::runtime_error("delivery pipeline stopped: " + step_error_msg_);
    out_free_.assign(Q_, 0);
    eof_count_ = 0;
    step_buffers_ = 0;
    step_error_ = 0;
    step_d2h_ms_ = 0;
    step_check_delivery_ = validate && cfg_.check_delivery && deliver;
    pre_d2h_ck_.assign((size_t)Q_ * R_, 0);
    delivered_ck_.assign((size_t)Q_ * R_, 0);
  }
  std::vector<hipEvent_t> ev(4 * (size_t)Q_);
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  unsigned long long* vstats = d_validate_.as<unsigned long long>();
  Elem* vprev = reinterpret_cast<Elem*>(d_validate_.as<uint8_t>() + 64);
  Elem* vlast = vprev + R_;
  std::vector<bool> has_prev(R_, false);
  if (validate) {
    HIP_CHECK(hipMemsetAsync(d_validate_.as(), 0, 64, s_compute_));
    HIP_CHECK(hipMemsetAsync(d_diag_.as(), 0, (size_t)Q_ * diag_stride() * 8, s_compute_));
  }
  if (cfg_.replan) {
    const double tp = now_ms();
    refresh_plan();
    st.plan_ms = now_ms() - tp;
  }

  auto wait_until = [&](const std::function<bool()>& ready) {
    std::unique_lock<std::mutex> lk(mu_);
    while (!cv_.wait_for(lk, std::chrono::milliseconds(100), [&] { return ready() || stop_; })) {
      if (exchange_) {  // a lost peer must fail the step, not hang it
        lk.unlock();
        wait_exchange_ok();
        lk.lock();
      }
    }
    if (stop_) throw std::runtime_error("delivery pipeline failed: " + step_error_msg_);
  };

  // Spill tiers (pinned DRAM, disk): a staging thread fills each round's HBM buffers ahead of the
  // round loop: the own cells into the receive slot and, at world > 1, the outgoing slices into the
  // round's send staging (peers only ever read device memory). Pinned DRAM is copied on an SDMA
  // engine of its own: a copy kernel (or hipMemcpyAsync, which runs as one) reading host memory
  // stalls the merge kernels beside it in the CU memory pipeline, while on the copy engines staging
  // overlaps delivery (the link's other direction) and the merge. The disk tier reads through
  // io_uring into the pinned chunk ring and copies to HBM on a stream of its own. Before reusing a
  // receive slot the thread waits for the merge that read it; before reusing a send staging parity,
  // for the exchange that sent it and for the peers' copies (Exchange::wait_sent). The round loop
  // waits for staged_round[q] instead of a stream dependency, then enqueues the exchange.
  const bool staged_send = W > 1 && spilled();
  const bool sdma_stage = spilled() && (disk_store() || (host_store() && sdma_h2d_));
  if (sdma_stage && disk_store() && !s_stage_) HIP_CHECK(hipStreamCreateWithFlags(&s_stage_, hipStreamNonBlocking));
  const int64_t xbase = xseq_;  // sequence number of this step's first exchange
  std::vector<char> staged_round(Q_, 0), merge_recorded(Q_, 0), xchg_recorded(Q_, 0);
  double stage_ms = 0;
  std::thread stage_thr;
  if (sdma_stage)
    stage_thr = std::thread([&] {
      try {
        HIP_CHECK(hipSetDevice(cfg_.device));
        SdmaEngine* eng = host_store() ? &SdmaEngine::for_device(cfg_.device) : nullptr;
        hsa_signal_t sig{};
        if (eng) sig = eng->make_signal();
        struct SigGuard {
          SdmaEngine* e;
          hsa_signal_t s;
          ~SigGuard() {
            if (e) e->destroy_signal(s);
          }
        } sig_guard{eng, sig};
        for (int q = 0; q < Q_; ++q) {
          const int slot = q % kSlots;
          if (q >= kSlots) {
            {
              std::unique_lock<std::mutex> lk(mu_);
              cv_.wait(lk, [&] { return merge_recorded[q - kSlots] != 0 || stop_; });
              if (stop_) break;
            }
            HIP_CHECK(hipEventSynchronize(merged_ev_[slot]));  // the slot's previous round is merged
          }
          if (staged_send && q >= 2) {  // send staging parity q & 1 was sent by exchange q-2
            {
              std::unique_lock<std::mutex> lk(mu_);
              cv_.wait(lk, [&] { return xchg_recorded[q - 2] != 0 || stop_; });
              if (stop_) break;
            }
            HIP_CHECK(hipEventSynchronize(sent_ev_[q & 1]));
            exchange_->wait_sent(xbase + q - 2);
          }
          const double ts = now_ms();
          const RoundPlan& rp = plans_[q];
          uint8_t* rbuf = recv_slots_[slot].as<uint8_t>();
          std::vector<CopyDesc> pieces;
          std::vector<DiskStore::Piece> dpieces;
          auto add = [&](int m, int64_t at, int64_t bytes, uint8_t* dst) {  // at: store offset of the bytes
            if (eng)
              pieces.push_back(CopyDesc{store_base_ + at, dst, bytes});
            else
              dpieces.push_back(DiskStore::Piece{m, at - mof_off_[m], bytes, dst});
          };
          for (int i = 0; i < R_; ++i)
            for (int j = 0; j < M; ++j) {
              const size_t x = ((size_t)me * R_ + i) * M + j;
              const int64_t cnt = rp.recv_cnt[x];
              if (cnt <= 0) continue;
              add(j, run_off_[j * W + me] + rp.self_beg[(size_t)i * M + j] * kTeraRecordBytes, cnt * kTeraRecordBytes,
                  rbuf + rp.recv_off[x]);
            }
          if (staged_send) {
            int64_t off = 0;
            for (int p = 0; p < W; ++p)
              for (const Span& sp : rp.send[p]) {  // span pointers are store_base_ + store offset
                const int64_t at = (int64_t)(sp.ptr - store_base_);
                const int m = (int)(std::upper_bound(mof_off_.begin(), mof_off_.end(), at) - mof_off_.begin()) - 1;
                add(m, at, sp.bytes, send_staging_[q & 1].as<uint8_t>() + off);
                off += sp.bytes;
              }
          }
          if (eng) {
            SdmaEngine::arm(sig, (int64_t)pieces.size());
            for (const CopyDesc& d : pieces) eng->copy_h2d(d.dst, d.src, (size_t)d.bytes, sig);
            SdmaEngine::wait(sig);
          } else {
            if (!dpieces.empty()) disk_->stage(dpieces, s_stage_);
            HIP_CHECK(hipStreamSynchronize(s_stage_));
          }
          std::lock_guard<std::mutex> g(mu_);
          staged_round[q] = 1;
          stage_ms += now_ms() - ts;
          cv_.notify_all();
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu_);
        if (!stop_) step_error_msg_ = std::string("H2D staging: ") + e.what();
        stop_ = true;
        cv_.notify_all();
      }
    });
  struct JoinGuard {
    std::thread& t;
    std::mutex& mu;
    std::condition_variable& cv;
    bool& stop;
    ~JoinGuard() {
      if (!t.joinable()) return;
      if (std::uncaught_exceptions() > 0) {  // the round loop failed: release the stager
        std::lock_guard<std::mutex> g(mu);
        stop = true;
        cv.notify_all();
      }
      t.join();
    }
  } stage_guard{stage_thr, mu_, cv_, stop_};

  // runs of round q, grouped by reducer: group i = cell (i, q) from every source map
  auto build_runs = [&](int q, std::vector<RunDesc>& runs, std::vector<int>& group_first) {
    const RoundPlan& rp = plans_[q];
    uint8_t* rbuf = staged() ? recv_slots_[q % kSlots].as<uint8_t>() : nullptr;
    runs.clear();
    group_first.assign(1, 0);
    runs.reserve((size_t)R_ * W * M);
    for (int i = 0; i < R_; ++i) {
      for (int s = 0; s < W; ++s)
        for (int j = 0; j < M; ++j) {
          const size_t x = ((size_t)s * R_ + i) * M + j;
          RunDesc d;
          d.nrec = rp.recv_cnt[x];
          d.nbytes = d.nrec * kTeraRecordBytes;
          d.offsets = nullptr;
          if (rp.recv_off[x] >= 0)
            d.base = rbuf + rp.recv_off[x];
          else  // own cell, read in place from the HBM store
            d.base = store_dev_base_ + run_off_[j * W + me] + rp.self_beg[(size_t)i * M + j] * kTeraRecordBytes;
          runs.push_back(d);
        }
      group_first.push_back((int)runs.size());
    }
  };
  // Runs read in place (HBM store, one rank): round q+1's cell planning is enqueued on the plan stream
  // right after round q's tiles, so it runs beside them instead of between them (+1.7 % device-only,
  // profiles/r3_kway_lookahead_ab.md).
  bool lookahead = false;
  DeviceMerger::KwayPlan next_plan;
  if (!staged() && merger_->kway_enabled()) {
    std::vector<RunDesc> r0;
    std::vector<int> g0;
    build_runs(0, r0, g0);
    if (merger_->kway_applicable(r0, g0)) {
      lookahead = true;
      next_plan = merger_->plan_kway(r0, g0, s_plan_);
    }
  }

  for (int q = 0; q < Q_; ++q) {
    trace::Range tr_round("uda.round");
    const int slot = q % kSlots;
    const RoundPlan& rp = plans_[q];
    uint8_t* rbuf = staged() ? recv_slots_[slot].as<uint8_t>() : nullptr;
    if (spilled())
      for (int i = 0; i < R_; ++i)
        for (int j = 0; j < M; ++j) st.bytes_h2d += rp.recv_cnt[((size_t)me * R_ + i) * M + j] * kTeraRecordBytes;
    if (staged_send) st.bytes_h2d += rp.send_bytes;
    if (sdma_stage) wait_until([&] { return staged_round[q] != 0; });
    if (staged()) {
      if (q >= kSlots) HIP_CHECK(hipStreamWaitEvent(s_comm_, merged_ev_[slot], 0));  // slot consumed
      HIP_CHECK(hipEventRecord(ev[4 * q + 0], s_comm_));
      if (spilled() && !sdma_stage) {  // pinned DRAM, copy-kernel staging (UDA_H2D_SDMA=0)
        if (staged_send && q >= 2) exchange_->wait_sent(xbase + q - 2);  // peers done with this parity
        launch_batched_copy(h2d_descs_[q].as<CopyDesc>(), h2d_n_[q], h2d_max_[q], s_comm_, h2d_blocks_);
      }
      if (W > 1) {
        if (staged_send) {
          exchange_->exchange(rp.staged_send, rp.staged_recv, s_comm_);
        } else {
          std::vector<std::vector<Span>> recv(W);
          for (int s = 0; s < W; ++s) {
            if (s == me) continue;
            for (int i = 0; i < R_; ++i)
              for (int j = 0; j < M; ++j) {
                const size_t x = ((size_t)s * R_ + i) * M + j;
                if (rp.recv_cnt[x] > 0) recv[s].push_back(Span{rbuf + rp.recv_off[x], rp.recv_cnt[x] * kTeraRecordBytes});
              }
          }
          exchange_->exchange(rp.send, recv, s_comm_);
        }
        ++xseq_;
        HIP_CHECK(hipEventRecord(sent_ev_[q & 1], s_comm_));
        {
          std::lock_guard<std::mutex> g(mu_);
          xchg_recorded[q] = 1;
        }
        cv_.notify_all();
        st.bytes_sent += rp.send_bytes;
      }
      HIP_CHECK(hipEventRecord(ev[4 * q + 1], s_comm_));
      HIP_CHECK(hipEventRecord(comm_ev_[slot], s_comm_));
      HIP_CHECK(hipStreamWaitEvent(s_compute_, comm_ev_[slot], 0));
    }
    std::vector<RunDesc> runs;
    std::vector<int> group_first;
    if (!lookahead) build_runs(q, runs, group_first);
    // output slot reuse: every D2H piece of round q-kSlots must have landed
    if (deliver && q >= kSlots) {
      const double tw = now_ms();
      wait_until([&] { return out_free_[q - kSlots] != 0; });
      st.wait_out_ms += now_ms() - tw;
    }
    unsigned long long* dg = d_diag_.as<unsigned long long>() + (size_t)q * diag_stride();
    // the merge's inputs as it is about to read them: received slices and own cells against their
    // plan-time checksums (the same checks after the merge tell a late write from a late read)
    auto check_inputs = [&](int at) {
      if (W > 1 && verify_n_[q] > 0) {
        launch_slice_checksums(d_verify_runs_[q].as<RunDesc>(), verify_n_[q], verify_max_nrec_[q],
                               d_verify_got_.as<unsigned long long>(), s_compute_);
        launch_count_mismatch(d_verify_got_.as<unsigned long long>(), d_verify_expect_[q].as<unsigned long long>(),
                              verify_n_[q], dg + at, s_compute_);
        if (at == 1)
          launch_count_mismatch(d_verify_got_.as<unsigned long long>(),
                                d_verify_expect_[q].as<unsigned long long>(), verify_n_[q], vstats + 2, s_compute_);
      }
      if (own_n_[q] > 0) {
        launch_slice_checksums(d_own_runs_[q].as<RunDesc>(), own_n_[q], own_max_nrec_[q],
                               d_verify_got_.as<unsigned long long>(), s_compute_);
        launch_count_mismatch(d_verify_got_.as<unsigned long long>(), d_own_expect_[q].as<unsigned long long>(),
                              own_n_[q], dg + at + 2, s_compute_);
      }
      HIP_CHECK(hipGetLastError());
    };
    if (validate) check_inputs(0);
    HIP_CHECK(hipEventRecord(ev[4 * q + 2], s_compute_));
    uint8_t* out = out_slots_[slot].as<uint8_t>();
    int64_t n = 0;
    if (lookahead) {  // this round was planned while the previous one merged; plan the next one now
      n = merger_->run_kway(next_plan, out, s_compute_);
      if (q + 1 < Q_) {
        build_runs(q + 1, runs, group_first);
        next_plan = merger_->plan_kway(runs, group_first, s_plan_);
      }
    } else {
      n = merger_->merge_fixed(runs, group_first, out, s_compute_);
    }
    HIP_CHECK(hipGetLastError());
    st.merge_passes = std::max(st.merge_passes, merger_->last_passes());
    if (validate) {
      int64_t goff = 0;
      for (int i = 0; i < R_; ++i) {
        const int64_t g = rp.group_recs[i];
        if (g > 0) {
          launch_validate_fixed(out + goff * kTeraRecordBytes, g, vprev + i, has_prev[i] ? 1 : 0, vlast + i, vstats,
                                s_compute_, dg + 4 + i);
          HIP_CHECK(hipMemcpyAsync(vprev + i, vlast + i, sizeof(Elem), hipMemcpyDeviceToDevice, s_compute_));
          has_prev[i] = true;
        }
        goff += g;
      }
      check_inputs(1);
    }
    HIP_CHECK(hipEventRecord(ev[4 * q + 3], s_compute_));
    HIP_CHECK(hipEventRecord(merged_ev_[slot], s_compute_));
    if (sdma_stage) {
      std::lock_guard<std::mutex> g(mu_);
      merge_recorded[q] = 1;
      cv_.notify_all();
    }
    st.records += n;
    if (deliver) {
      {
        std::lock_guard<std::mutex> g(mu_);
        round_q_.push_back(RoundOut{q, slot, rp.group_recs});
      }
      cv_.notify_all();
    }
  }
  if (deliver) wait_until([&] { return eof_count_ == R_; });
  if (exchange_) exchange_->wait(s_comm_);
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  HIP_CHECK(hipStreamSynchronize(s_comm_));
  HIP_CHECK(hipStreamSynchronize(s_copy_));
  if (stage_thr.joinable()) stage_thr.join();
  // every rank's pulls from this rank's memory are done before any rank reuses or frees it
  if (exchange_) exchange_->quiesce();
  st.wall_ms = now_ms() - t0;
  st.stage_ms = stage_ms;
  for (int q = 0; q < Q_; ++q) {
    float a = 0, b = 0;
    if (staged() && hipEventElapsedTime(&a, ev[4 * q + 0], ev[4 * q + 1]) == hipSuccess) st.comm_ms += a;
    if (hipEventElapsedTime(&b, ev[4 * q + 2], ev[4 * q + 3]) == hipSuccess) st.merge_ms += b;
    st.round_comm_ms.push_back(a);
    st.round_merge_ms.push_back(b);
  }
  static const bool round_trace = std::getenv("UDA_ROUND_TRACE") != nullptr;  // tools: per-round timeline
  if (round_trace && staged()) {
    std::string line = "[round trace ms: comm start-end | merge start-end]";
    for (int q = 0; q < Q_; ++q) {
      float t[4] = {0, 0, 0, 0};
      for (int k = 0; k < 4; ++k) (void)hipEventElapsedTime(&t[k], ev[0], ev[4 * q + k]);
      char b[96];
      snprintf(b, sizeof(b), " q%d %.0f-%.0f|%.0f-%.0f", q, t[0], t[1], t[2], t[3]);
      line += b;
    }
    fprintf(stderr, "%s\n", line.c_str());
  }
  for (auto e : ev) (void)hipEventDestroy(e);
  st.d2h_ms = step_d2h_ms_;
  st.bytes_in = st.records * kTeraRecordBytes;
  st.buffers = step_buffers_;
  if (validate) {
    unsigned long long v[3];
    HIP_CHECK(hipMemcpy(v, vstats, sizeof(v), hipMemcpyDeviceToHost));
    st.order_errors = (int64_t)v[0];
    st.checksum = v[1];
    st.exchange_errors = W > 1 ? (int64_t)v[2] : 0;
    localize_mismatch(st);
  }
  st.bad_layout = merger_->bad_layout();
  if (step_error_) throw std::runtime_error("delivery sink reported error " + std::to_string(step_error_));
  return st;
}

}  // namespace gpu
}  // namespace uda
