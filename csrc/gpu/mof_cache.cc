// Provider HBM store for MOF files. See mof_cache.h.
#include "mof_cache.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "device_engine.h"
#include "sdma.h"
#include "uda/aio.h"
#include "uda/log.h"

namespace uda {
namespace gpu {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int64_t align_io(int64_t v) { return (v + kAioAlignment - 1) / kAioAlignment * kAioAlignment; }
}  // namespace

MofCache::MofCache(const Options& o) : opt_(o) {
  opt_.chunk_bytes = align_io(std::max<int64_t>(opt_.chunk_bytes, 1 << 20));
  opt_.chunks = std::max(2, opt_.chunks);
  if (!enabled()) return;
  per_device_ = opt_.capacity / (int64_t)opt_.devices.size();
  for (int d : opt_.devices) used_[d] = 0;
}

MofCache::~MofCache() {
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : entries_)
      if (!kv.second->loading) free_entry(kv.second.get());
    entries_.clear();
  }
  std::lock_guard<std::mutex> g(load_mu_);
  if (aio_) aio_->drain();
  for (auto e : ev_) (void)hipEventDestroy(e);
  for (auto s : streams_)
    if (s) (void)hipStreamDestroy(s);
  if (ring_) pinned_host_free(ring_);
}

void MofCache::free_entry(Entry* e) {
  if (e->dptr) (void)hipFree(e->dptr);
  e->dptr = nullptr;
}

bool MofCache::make_room(int device, int64_t bytes, double now) {
  if (bytes > per_device_) return false;
  while (used_[device] + bytes > per_device_) {
    std::map<std::string, std::shared_ptr<Entry>>::iterator victim = entries_.end();
    for (auto it = entries_.begin(); it != entries_.end(); ++it) {
      Entry& e = *it->second;
      if (e.device != device || e.loading) continue;
      if (!e.job_done && now - e.last_served < opt_.lease_s) continue;  // a reducer may still read it
      if (victim == entries_.end() || e.last_served < victim->second->last_served) victim = it;
    }
    if (victim == entries_.end()) return false;
    UDA_LOG(kDebug, "provider HBM store: evicting %s (%ld bytes)", victim->first.c_str(), (long)victim->second->len);
    used_[device] -= victim->second->len;
    free_entry(victim->second.get());
    entries_.erase(victim);
    st_.evictions++;
  }
  return true;
}

bool MofCache::acquire(const std::string& job, const std::string& path, Ref* out, std::string* why) {
  if (!enabled()) {
    if (why) *why = "provider HBM store disabled";
    return false;
  }
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    auto it = entries_.find(path);
    if (it == entries_.end()) break;
    std::shared_ptr<Entry> e = it->second;
    if (e->loading) {
      cv_.wait(lk);
      continue;
    }
    e->last_served = now_s();
    st_.hits++;
    out->data = static_cast<const uint8_t*>(e->dptr);
    out->len = e->len;
    out->device = e->device;
    out->ipc = e->ipc;
    return true;
  }
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0) {
    if (why) *why = "cannot stat " + path + ": " + strerror(errno);
    st_.declined++;
    return false;
  }
  const int64_t len = (int64_t)sb.st_size;
  int device = opt_.devices[0];
  for (int d : opt_.devices)
    if (per_device_ - used_[d] > per_device_ - used_[device]) device = d;
  if (!make_room(device, std::max<int64_t>(len, 1), now_s())) {
    if (why) *why = "provider HBM budget exhausted (all resident MOFs leased)";
    st_.declined++;
    return false;
  }
  auto e = std::make_shared<Entry>();
  e->job = job;
  e->device = device;
  e->len = len;
  used_[device] += std::max<int64_t>(len, 1);
  entries_[path] = e;
  lk.unlock();
  const double t0 = now_s();
  try {
    load(path, e.get());
  } catch (const std::exception& ex) {
    lk.lock();
    used_[device] -= std::max<int64_t>(len, 1);
    free_entry(e.get());
    entries_.erase(path);
    st_.declined++;
    cv_.notify_all();
    if (why) *why = ex.what();
    UDA_LOG(kWarn, "provider HBM store: loading %s failed: %s", path.c_str(), ex.what());
    return false;
  }
  lk.lock();
  e->loading = false;
  e->last_served = now_s();
  st_.loads++;
  st_.bytes_loaded += len;
  st_.load_ms += (now_s() - t0) * 1000.0;
  cv_.notify_all();
  out->data = static_cast<const uint8_t*>(e->dptr);
  out->len = e->len;
  out->device = e->device;
  out->ipc = e->ipc;
  return true;
}

// Whole file -> HBM: reads of chunk_bytes (O_DIRECT, 4 KiB aligned) into the pinned ring with up to
// `chunks` in flight; each landed chunk is copied H2D on the device's stream, and its ring slot is
// reused once that copy finished.
void MofCache::load(const std::string& path, Entry* e) {
  std::lock_guard<std::mutex> g(load_mu_);
  const int dev_index = (int)(std::find(opt_.devices.begin(), opt_.devices.end(), e->device) - opt_.devices.begin());
  HIP_CHECK(hipSetDevice(e->device));
  if (!aio_) {
    AsyncIO::Options ao;
    ao.threads = 4;
    ao.queue_depth = 2 * opt_.chunks;
    aio_ = AsyncIO::create(ao);
    ring_ = static_cast<uint8_t*>(
        hip_host_alloc_on_node((size_t)(opt_.chunk_bytes * opt_.chunks), device_numa_node(opt_.devices[0])));
    ev_.resize((size_t)opt_.chunks, nullptr);
    for (auto& ev : ev_) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    streams_.assign(opt_.devices.size(), nullptr);
  }
  if (!streams_[(size_t)dev_index]) HIP_CHECK(hipStreamCreateWithFlags(&streams_[(size_t)dev_index], hipStreamNonBlocking));
  hipStream_t s = streams_[(size_t)dev_index];
  HIP_CHECK(hipMalloc(&e->dptr, ipc_safe_bytes((size_t)std::max<int64_t>(e->len, 1))));
  e->ipc = ipc_export(e->dptr);
  bool direct = opt_.odirect;
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC | (direct ? O_DIRECT : 0));
  if (fd < 0 && direct) {
    direct = false;
    fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  }
  if (fd < 0) throw std::runtime_error("cannot open " + path + ": " + strerror(errno));
  struct FdGuard {
    int fd;
    ~FdGuard() { ::close(fd); }
  } fg{fd};
  const int64_t C = opt_.chunk_bytes, n = (e->len + C - 1) / C;
  const int K = opt_.chunks;
  std::vector<int64_t> result((size_t)n, 0);
  std::vector<char> done((size_t)n, 0);
  std::vector<char> pending((size_t)K, 0);
  std::mutex m;
  std::condition_variable c;
  int64_t next_submit = 0, next_finish = 0;
  try {
    while (next_finish < n) {
      while (next_submit < n && next_submit - next_finish < K) {
        const int slot = (int)(next_submit % K);
        if (pending[(size_t)slot]) {  // the slot's previous H2D must have read it
          HIP_CHECK(hipEventSynchronize(ev_[(size_t)slot]));
          pending[(size_t)slot] = 0;
        }
        const int64_t off = next_submit * C;
        const int64_t want = std::min(C, e->len - off);
        const int64_t i = next_submit;
        aio_->read(fd, off, direct ? align_io(want) : want, ring_ + (int64_t)slot * C, [&, i](int64_t r) {
          std::lock_guard<std::mutex> lg(m);
          result[(size_t)i] = r;
          done[(size_t)i] = 1;
          c.notify_all();
        });
        ++next_submit;
      }
      {
        std::unique_lock<std::mutex> lk(m);
        c.wait(lk, [&] { return done[(size_t)next_finish] != 0; });
      }
      const int64_t off = next_finish * C;
      const int64_t want = std::min(C, e->len - off);
      if (result[(size_t)next_finish] < want)
        throw std::runtime_error("short read from " + path + " at " + std::to_string(off));
      const int slot = (int)(next_finish % K);
      HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(e->dptr) + off, ring_ + (int64_t)slot * C, (size_t)want,
                               hipMemcpyHostToDevice, s));
      HIP_CHECK(hipEventRecord(ev_[(size_t)slot], s));
      pending[(size_t)slot] = 1;
      ++next_finish;
    }
    HIP_CHECK(hipStreamSynchronize(s));
  } catch (...) {
    aio_->drain();  // no read may land in the ring after we leave
    (void)hipStreamSynchronize(s);
    throw;
  }
}

void MofCache::job_over(const std::string& job) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = entries_.begin(); it != entries_.end();) {
    Entry& e = *it->second;
    if (e.job == job && !e.loading) {
      used_[e.device] -= std::max<int64_t>(e.len, 1);
      free_entry(&e);
      st_.evictions++;
      it = entries_.erase(it);
    } else {
      if (e.job == job) e.job_done = true;
      ++it;
    }
  }
}

MofCache::Stats MofCache::stats() {
  std::lock_guard<std::mutex> g(mu_);
  Stats s = st_;
  s.resident_bytes = 0;
  for (auto& kv : used_) s.resident_bytes += kv.second;
  return s;
}

}  // namespace gpu
}  // namespace uda
