// Provider HBM store for MOF files. See mof_cache.h.
#include "mof_cache.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "device_engine.h"
#include "sdma.h"
#include "uda/aio.h"
#include "uda/fault.h"
#include "uda/log.h"
#include "uda/node_registry.h"
#include "uda/start_trace.h"
#include "uda/thread_name.h"

namespace uda {
namespace gpu {

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int64_t align_io(int64_t v) { return (v + kAioAlignment - 1) / kAioAlignment * kAioAlignment; }

// holder id "<node>:<pid>:<start ticks>:<task>" (reducer_holder_id in device_ptr.h)
bool holder_alive(const std::string& h, double last, double now, double lease_s) {
  const size_t a = h.find(':');
  const size_t b = a == std::string::npos ? a : h.find(':', a + 1);
  const size_t c = b == std::string::npos ? b : h.find(':', b + 1);
  if (c == std::string::npos) return now - last < lease_s;  // not ours to check: lease only
  if (h.compare(0, a, node_id()) != 0) return now - last < lease_s;  // another node
  const int pid = std::atoi(h.substr(a + 1, b - a - 1).c_str());
  const uint64_t start = std::strtoull(h.substr(b + 1, c - b - 1).c_str(), nullptr, 10);
  return process_running(pid, start);
}
}  // namespace

static double boot_ms() {
  timespec ts{};
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6;
}

struct MofCache::Loader {
  enum State { kFree = 0, kReading = 1, kCopying = 2 };
  struct Slot {
    State state = kFree;
    std::shared_ptr<Entry> e;
    int64_t off = 0, len = 0, result = 0;
    bool read_done = false;
    hsa_signal_t sig{};
    hipEvent_t ev = nullptr;
    int parts = 0;  // disk reads of this chunk still in flight
  };
  int device = 0;
  std::thread thr;
  std::vector<std::thread> openers;  // allocate HBM and open the file of new entries (never stall the reads)
  std::condition_variable cv;  // with MofCache::mu_
  std::condition_variable ocv; // opener: new pending entries (with MofCache::mu_)
  bool stop = false;
  std::deque<std::shared_ptr<Entry>> pending;  // to allocate + open (opener thread)
  int opening = 0;                             // taken by the opener, not yet active
  std::deque<std::shared_ptr<Entry>> active;   // unread bytes left, read in turn
  std::vector<Slot> slots;
  std::unique_ptr<AsyncIO> aio;
  // Buffered reads of files already in the page cache (Options::cached_read) are memory copies, done by
  // this pool of threads (io_uring completes them inline on its two submitting threads: ~21 GB/s per GPU)
  std::vector<std::thread> readers;
  std::deque<std::function<void()>> rq;
  std::condition_variable rcv;  // with rmu
  std::mutex rmu;
  bool rstop = false;
  uint8_t* ring = nullptr;
  SdmaEngine* sdma = nullptr;
  hipStream_t stream = nullptr;
  bool ready = false;
  bool failed = false;  // setup failed: every entry of this device is declined (mu_)
  std::string setup_error;
};

MofCache::MofCache(const Options& o) : opt_(o) {
  // tuning A/Bs of the load path (tools/gpu_run.py): chunk size and chunks in flight per loader
  if (const char* e = std::getenv("UDA_STORE_CHUNK_MB")) opt_.chunk_bytes = std::atoll(e) << 20;
  if (const char* e = std::getenv("UDA_STORE_CHUNKS")) opt_.chunks = std::atoi(e);
  opt_.chunk_bytes = align_io(std::max<int64_t>(opt_.chunk_bytes, 1 << 20));
  opt_.chunks = std::max(2, opt_.chunks);
  if (const char* e = std::getenv("UDA_STORE_READ_MB")) opt_.read_bytes = std::atoll(e) << 20;
  if (const char* e = std::getenv("UDA_STORE_EAGER_EXPORT")) eager_export_ = std::atoi(e) != 0;  // A/B
  opt_.read_bytes = opt_.read_bytes <= 0 ? opt_.chunk_bytes
                                         : align_io(std::min(opt_.read_bytes, opt_.chunk_bytes));
  if (!enabled()) return;
  per_device_ = opt_.capacity / (int64_t)opt_.devices.size();
  for (int d : opt_.devices) used_[d] = 0;
}

MofCache::Loader* MofCache::loader_locked(int device) {
  std::unique_ptr<Loader>& L = loaders_[device];
  if (!L) {
    L.reset(new Loader);
    L->device = device;
    Loader* lp = L.get();
    L->thr = std::thread([this, lp] { name_thread("uda-store-load"); loader_main(lp); });
    int n = 1;  // A/B: UDA_STORE_OPENERS entries allocated + exported + opened at once
    if (const char* e = std::getenv("UDA_STORE_OPENERS")) n = std::max(1, std::min(16, std::atoi(e)));
    for (int i = 0; i < n; ++i) L->openers.emplace_back([this, lp] { name_thread("uda-store-open"); opener_main(lp); });
  }
  return L.get();
}

void MofCache::start_loaders() {
  if (!enabled()) return;
  std::lock_guard<std::mutex> g(mu_);
  for (int d : opt_.devices) (void)loader_locked(d);
}

MofCache::~MofCache() {
  std::vector<std::unique_ptr<Loader>> ls;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : loaders_) {
      kv.second->stop = true;
      kv.second->cv.notify_all();
    }
  }
  for (auto& kv : loaders_) {
    kv.second->ocv.notify_all();
    for (auto& t : kv.second->openers)
      if (t.joinable()) t.join();
    if (kv.second->thr.joinable()) kv.second->thr.join();
  }
  std::lock_guard<std::mutex> g(mu_);
  entries_.clear();
  loaders_.clear();
}

MofCache::Ref MofCache::ref_of(const Entry& e) const {
  Ref r;
  r.data = e.dptr;
  r.len = e.len;
  r.device = e.device;
  r.ipc = e.ipc;
  return r;
}

bool MofCache::evictable(Entry& e, double now) {
  if (e.loading) return false;
  for (auto it = e.holders.begin(); it != e.holders.end();) {
    if (holder_alive(it->first, it->second.second, now, opt_.lease_s)) {
      ++it;
    } else {
      UDA_LOG(kInfo, "provider HBM store: holder %s of %s is gone; its references dropped", it->first.c_str(),
              e.path.c_str());
      st_.holders_reaped++;
      it = e.holders.erase(it);
    }
  }
  return e.job_done || e.holders.empty();
}

void MofCache::erase_entry(const std::string& path) {
  auto it = entries_.find(path);
  if (it == entries_.end()) return;
  used_[it->second->device] -= std::max<int64_t>(it->second->len, 1);
  entries_.erase(it);  // the HBM goes when the last in-flight chunk of it is done
}

bool MofCache::make_room(int device, int64_t bytes, double now, const std::string& job) {
  if (bytes > per_device_) return false;
  while (used_[device] + bytes > per_device_) {
    // finished jobs first, then unreferenced entries, least recently served first; an entry of the same
    // job (still running) only once idle (Options::idle_evict_s)
    std::shared_ptr<Entry> victim;
    for (auto& kv : entries_) {
      Entry& e = *kv.second;
      const int64_t reaped = st_.holders_reaped;
      if (e.device != device || !evictable(e, now)) continue;
      if (!e.job_done && e.job == job && opt_.idle_evict_s > 0 && now - e.last_served < opt_.idle_evict_s &&
          st_.holders_reaped == reaped)  // (an entry whose holder just turned out dead is fair game)
        continue;
      if (!victim || (e.job_done && !victim->job_done) ||
          (e.job_done == victim->job_done && e.last_served < victim->last_served))
        victim = kv.second;
    }
    if (!victim) return false;
    UDA_LOG(kDebug, "provider HBM store: evicting %s (%ld bytes)", victim->path.c_str(), (long)victim->len);
    erase_entry(victim->path);
    st_.evictions++;
  }
  return true;
}

void MofCache::collect_ready(Entry& e, std::vector<Fire>* fire) {
  for (auto it = e.waiters.begin(); it != e.waiters.end();) {
    if (it->need_end <= e.landed || !e.loading) {  // (a whole-file waiter asks past the end)
      fire->push_back(Fire{std::move(it->ready), true, ref_of(e), std::string()});
      it = e.waiters.erase(it);
    } else {
      ++it;
    }
  }
}

void MofCache::fail_entry(Entry& e, const std::string& why, std::vector<Fire>* fire) {
  if (e.failed) return;
  e.failed = true;
  e.loading = false;
  e.error = why;
  UDA_LOG(kWarn, "provider HBM store: loading %s failed: %s", e.path.c_str(), why.c_str());
  for (auto& w : e.waiters) fire->push_back(Fire{std::move(w.ready), false, Ref(), why});
  e.waiters.clear();
  st_.declined++;
  if (e.fd >= 0 && e.reads_in_flight == 0) {
    ::close(e.fd);
    e.fd = -1;
  }
  auto it = entries_.find(e.path);
  if (it != entries_.end() && it->second.get() == &e) erase_entry(e.path);
}

bool MofCache::acquire_async(const std::string& job, const std::string& path, const std::string& holder,
                             int64_t need_end, Ready ready, std::string* why) {
  if (!enabled()) {
    if (why) *why = "provider HBM store disabled";
    return false;
  }
  start_trace("store_acquire_begin", 0);
  std::unique_lock<std::mutex> lk(mu_);
  start_trace("store_acquire_locked", 0);
  const double now = now_s();
  auto it = entries_.find(path);
  if (it != entries_.end()) {
    std::shared_ptr<Entry> e = it->second;
    e->last_served = now;
    auto& h = e->holders[holder];
    h.first++;
    h.second = now;
    st_.hits++;
    if (e->landed >= need_end || !e->loading) {
      const Ref r = ref_of(*e);
      lk.unlock();
      ready(true, r, std::string());
    } else {
      e->waiters.push_back(Waiter{need_end, std::move(ready)});
    }
    return true;
  }
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0) {
    if (why) *why = "cannot stat " + path + ": " + strerror(errno);
    st_.declined++;
    return false;
  }
  const int64_t len = (int64_t)sb.st_size;
  // a device whose loader could not be set up (no HIP device, no pinned memory, ...) takes nothing:
  // its entries would never load and their waiters never be answered
  int device = -1;
  std::string dead;
  for (int d : opt_.devices) {
    auto l = loaders_.find(d);
    if (l != loaders_.end() && l->second->failed) {
      dead = l->second->setup_error;
      continue;
    }
    if (device < 0 || per_device_ - used_[d] > per_device_ - used_[device]) device = d;
  }
  if (device < 0) {
    if (why) *why = "provider HBM store unavailable: " + dead;
    st_.declined++;
    return false;
  }
  if (!make_room(device, std::max<int64_t>(len, 1), now, job)) {
    if (why) *why = "provider HBM budget exhausted (every resident MOF is held by a reducer or recently served to its job)";
    st_.declined++;
    return false;
  }
  auto e = std::make_shared<Entry>();
  e->job = job;
  e->path = path;
  e->device = device;
  e->len = len;
  e->last_served = e->t_start = now;
  if (st_.first_miss_boot_ms == 0) st_.first_miss_boot_ms = boot_ms();
  e->holders[holder] = {1, now};
  e->waiters.push_back(Waiter{need_end, std::move(ready)});
  used_[device] += std::max<int64_t>(len, 1);
  entries_[path] = e;
  Loader* L = loader_locked(device);
  L->pending.push_back(e);
  L->ocv.notify_all();
  return true;
}

IpcExport MofCache::export_of(const std::string& path) {
  std::shared_ptr<Entry> e;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = entries_.find(path);
    if (it == entries_.end() || it->second->failed || !it->second->dptr) {
      IpcExport none;
      none.handle_hex = "-";
      return none;
    }
    e = it->second;
    if (e->exported) return e->ipc;
  }
  std::lock_guard<std::mutex> eg(e->export_mu);  // the entry (and its memory) lives while `e` is held
  {
    std::lock_guard<std::mutex> g(mu_);
    if (e->exported) return e->ipc;
  }
  const double t0 = now_s();
  IpcExport x = ipc_export(e->dptr);
  std::lock_guard<std::mutex> g(mu_);
  st_.open_export_ms += (now_s() - t0) * 1000.0;
  e->ipc = x;
  e->exported = true;
  return x;
}

bool MofCache::acquire(const std::string& job, const std::string& path, const std::string& holder, Ref* out,
                       std::string* why) {
  std::mutex m;
  std::condition_variable c;
  bool done = false, ok = false;
  std::string err;
  if (!acquire_async(job, path, holder, INT64_MAX / 2, [&](bool k, const Ref& r, const std::string& w) {
        std::lock_guard<std::mutex> g(m);
        ok = k;
        if (k) *out = r;
        err = w;
        done = true;
        c.notify_all();
      }, why))
    return false;
  std::unique_lock<std::mutex> lk(m);
  c.wait(lk, [&] { return done; });
  if (!ok && why) *why = err;
  return ok;
}

void MofCache::release(const std::string& path, const std::string& holder) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = entries_.find(path);
  if (it == entries_.end()) return;
  auto h = it->second->holders.find(holder);
  if (h == it->second->holders.end()) return;
  st_.releases++;
  if (--h->second.first <= 0) it->second->holders.erase(h);
}

void MofCache::release_holder(const std::string& job, const std::string& holder) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : entries_) {
    Entry& e = *kv.second;
    if (job != "*" && e.job != job) continue;
    auto h = e.holders.find(holder);
    if (h == e.holders.end()) continue;
    st_.releases += h->second.first;
    e.holders.erase(h);
  }
}

void MofCache::job_over(const std::string& job) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> drop;
  for (auto& kv : entries_) {
    Entry& e = *kv.second;
    if (e.job != job) continue;
    e.job_done = true;
    if (!e.loading) drop.push_back(kv.first);
  }
  for (const auto& p : drop) {
    erase_entry(p);
    st_.evictions++;
  }
}

MofCache::Stats MofCache::stats() {
  std::lock_guard<std::mutex> g(mu_);
  Stats s = st_;
  s.resident_bytes = 0;
  for (auto& kv : used_) s.resident_bytes += kv.second;
  s.holders = 0;
  for (auto& kv : entries_)
    for (auto& h : kv.second->holders) s.holders += h.second.first;
  if (busy_loaders_ > 0) s.load_wall_ms += (now_s() - busy_since_) * 1000.0;
  return s;
}

// A loader's opener thread: HBM allocation (resident in the HBM budget), IPC export and the file of
// every new entry, so the reads of files already open never wait behind them (a 1.3 GB hipMalloc +
// export takes milliseconds; 32 of them serialized in the read loop cost the first step a second).
namespace {
// Share of a file's pages in the page cache (mincore over a read-only mapping); 0 if unknown.
double page_cache_share(const std::string& path, int64_t len) {
  if (len <= 0) return 0;
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  void* m = ::mmap(nullptr, (size_t)len, PROT_READ, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return 0;
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const size_t n = ((size_t)len + pg - 1) / pg;
  std::vector<unsigned char> v(n);
  size_t in = 0;
  if (::mincore(m, (size_t)len, v.data()) == 0)
    for (unsigned char c : v) in += c & 1;
  ::munmap(m, (size_t)len);
  return (double)in / (double)n;
}
}  // namespace

void MofCache::opener_main(Loader* L) {
  (void)hipSetDevice(L->device);
  std::vector<Fire> fire;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    L->ocv.wait(lk, [&] { return L->stop || !L->pending.empty(); });
    if (L->pending.empty()) return;  // stopped and drained
    std::shared_ptr<Entry> e = L->pending.front();
    L->pending.pop_front();
    ++L->opening;
    std::string err = L->stop ? "provider HBM store stopped" : "";
    std::unique_ptr<DeviceBuffer> mem;
    int fd = -1;
    bool direct = opt_.odirect;
    IpcExport ipc;
    lk.unlock();
    const double t0 = now_s();
    double t_alloc = t0, t_export = t0;
    if (err.empty()) {
      try {
        mem.reset(new DeviceBuffer((size_t)std::max<int64_t>(e->len, 1), /*resident=*/true));
        t_alloc = now_s();
        ipc.handle_hex = "-";  // exported on first need (export_of)
        ipc.base = mem->as<uint8_t>();
        if (eager_export_) ipc = ipc_export(mem->as<uint8_t>());
        t_export = now_s();
        // Map outputs written moments ago are still in the page cache: O_DIRECT would read them from the
        // disk again (the node's 32-file interleaved rate, 15-21 GB/s on the GPU boxes) instead of copying
        // them out of memory. The reference reads every MOF with O_DIRECT (IndexInfo.cc:304-335).
        if (direct && opt_.cached_read && page_cache_share(e->path, e->len) >= 0.9) {
          direct = false;
          std::lock_guard<std::mutex> g(mu_);
          st_.cached_reads++;
        }
        fd = ::open(e->path.c_str(), O_RDONLY | O_CLOEXEC | (direct ? O_DIRECT : 0));
        if (fd < 0 && direct) {
          direct = false;
          fd = ::open(e->path.c_str(), O_RDONLY | O_CLOEXEC);
        }
        if (fd < 0) err = "cannot open " + e->path + ": " + strerror(errno);
      } catch (const std::exception& ex) {
        err = ex.what();
      }
    }
    const double dt = now_s() - t0;
    lk.lock();
    --L->opening;
    st_.open_ms += dt * 1000.0;
    if (t_alloc > t0) {
      st_.open_alloc_ms += (t_alloc - t0) * 1000.0;
      st_.open_export_ms += (t_export - t_alloc) * 1000.0;
      st_.open_file_ms += (t0 + dt - t_export) * 1000.0;
      st_.open_file_max_ms = std::max(st_.open_file_max_ms, (t0 + dt - t_export) * 1000.0);
    }
    if (err.empty() && L->failed) err = "provider HBM store loader failed: " + L->setup_error;
    if (!err.empty() || e->failed) {
      if (fd >= 0) ::close(fd);
      fail_entry(*e, err.empty() ? e->error : err, &fire);
    } else {
      e->mem = std::move(mem);
      e->dptr = e->mem->as<uint8_t>();
      e->ipc = ipc;
      e->exported = eager_export_;
      e->fd = fd;
      e->direct = direct;
      if (e->len == 0) {
        e->loading = false;
        collect_ready(*e, &fire);
      } else {
        L->active.push_back(e);
      }
      L->cv.notify_all();
    }
    if (!fire.empty()) {
      lk.unlock();
      for (Fire& f : fire) f.ready(f.ok, f.ref, f.why);
      fire.clear();
      lk.lock();
    }
  }
}

// One loader per GPU: O_DIRECT chunk reads round-robin over the files being loaded, SDMA H2D of every
// landed chunk, and the readiness of each file's prefix.
void MofCache::loader_main(Loader* L) {
  const int C_slots = opt_.chunks;
  const int64_t C = opt_.chunk_bytes;
  std::vector<Fire> fire;
  try {
    if (fault_hit("STORE_SETUP")) throw std::runtime_error("injected provider HBM store setup failure");
    const int node = device_numa_node(L->device);
    bind_thread_to_numa(node);
    HIP_CHECK(hipSetDevice(L->device));
    AsyncIO::Options ao;
    ao.threads = 2;
    if (const char* e = std::getenv("UDA_STORE_AIO_THREADS")) ao.threads = std::max(1, std::atoi(e));
    ao.queue_depth = 2 * C_slots * (int)((C + opt_.read_bytes - 1) / opt_.read_bytes);
    L->aio = AsyncIO::create(ao);
    int nreaders = 8;
    if (const char* e = std::getenv("UDA_STORE_READERS")) nreaders = std::max(1, std::min(32, std::atoi(e)));
    for (int i = 0; i < nreaders; ++i)
      L->readers.emplace_back([L, node] {
        name_thread("uda-store-read");
        bind_thread_to_numa(node);
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> g(L->rmu);
            L->rcv.wait(g, [&] { return L->rstop || !L->rq.empty(); });
            if (L->rq.empty()) return;
            job = std::move(L->rq.front());
            L->rq.pop_front();
          }
          job();
        }
      });
    L->ring = static_cast<uint8_t*>(pinned_host_alloc((size_t)(C * C_slots), node));
    try {
      const char* h2d = std::getenv("UDA_STORE_H2D");  // A/B: "blit" copies chunks with hipMemcpyAsync
      L->sdma = h2d && std::string(h2d) == "blit" ? nullptr : &SdmaEngine::for_device(L->device);
      if (L->sdma) {
        // the runtime creates an SDMA engine's queue at its first copy (~150 ms): take that now, not at the
        // first chunk of the first wave -- the loader issues copies holding mu_, and every descriptor fetch
        // of the node (the daemon's control channel) waited behind it (UDA_START_TRACE: a 173 ms stall)
        void* scratch = nullptr;
        HIP_CHECK(hipMalloc(&scratch, 4096));
        try {
          L->sdma->warm(scratch);
        } catch (...) {
          (void)hipFree(scratch);
          throw;
        }
        HIP_CHECK(hipFree(scratch));
      }
    } catch (const std::exception& ex) {
      UDA_LOG(kWarn, "provider HBM store: no SDMA engine on device %d (%s); hipMemcpyAsync", L->device, ex.what());
      L->sdma = nullptr;
    }
    L->slots.resize((size_t)C_slots);
    for (auto& s : L->slots) {
      if (L->sdma) {
        s.sig = L->sdma->make_signal();
        SdmaEngine::arm(s.sig, 0);
      } else {
        HIP_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
      }
    }
    if (!L->sdma) HIP_CHECK(hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking));
    L->ready = true;
  } catch (const std::exception& ex) {
    L->setup_error = ex.what();
  }

  std::unique_lock<std::mutex> lk(mu_);
  if (!L->ready) {
    // the device cannot load files: decline everything queued on it (the reducers fetch the bytes
    // instead) and every later request for it (acquire_async skips a failed loader); the slot table may
    // be empty and the I/O ring null, so nothing below may run
    UDA_LOG(kWarn, "provider HBM store: loader of device %d failed to start: %s", L->device, L->setup_error.c_str());
    L->failed = true;
    for (auto& e : L->active) fail_entry(*e, "provider HBM store loader failed: " + L->setup_error, &fire);
    L->active.clear();
    for (auto& e : L->pending) fail_entry(*e, "provider HBM store loader failed: " + L->setup_error, &fire);
    L->pending.clear();
    lk.unlock();
    for (Fire& f : fire) f.ready(f.ok, f.ref, f.why);
    if (L->aio) L->aio->drain();
    {
      std::lock_guard<std::mutex> g(L->rmu);
      L->rstop = true;
      L->rcv.notify_all();
    }
    for (auto& t : L->readers) t.join();
    for (auto& sl : L->slots) {
      if (L->sdma && sl.sig.handle) L->sdma->destroy_signal(sl.sig);
      if (sl.ev) (void)hipEventDestroy(sl.ev);
    }
    if (L->stream) (void)hipStreamDestroy(L->stream);
    if (L->ring) pinned_host_free(L->ring);
    L->ring = nullptr;
    return;
  }
  bool was_busy = false;
  for (;;) {
    if (L->stop) {  // the store is going away: nothing new starts, loads in progress fail
      for (auto& e : L->active) fail_entry(*e, "provider HBM store stopped", &fire);
      L->active.clear();
    }
    // ---- landed reads: issue their H2D copies
    for (int i = 0; i < C_slots; ++i) {
      Loader::Slot& s = L->slots[(size_t)i];
      if (s.state != Loader::kReading || !s.read_done) continue;
      Entry& e = *s.e;
      if (e.failed || s.result < s.len) {
        if (!e.failed) fail_entry(e, "short read from " + e.path + " at " + std::to_string(s.off), &fire);
        if (--e.reads_in_flight == 0 && e.fd >= 0 && e.failed) {
          ::close(e.fd);
          e.fd = -1;
        }
        s = Loader::Slot{Loader::kFree, nullptr, 0, 0, 0, false, s.sig, s.ev};
        continue;
      }
      try {
        if (L->sdma) {
          SdmaEngine::arm(s.sig, 1);
          L->sdma->copy_h2d(const_cast<uint8_t*>(e.dptr) + s.off, L->ring + (int64_t)i * C, (size_t)s.len, s.sig);
        } else {
          HIP_CHECK(hipMemcpyAsync(const_cast<uint8_t*>(e.dptr) + s.off, L->ring + (int64_t)i * C, (size_t)s.len,
                                   hipMemcpyHostToDevice, L->stream));
          HIP_CHECK(hipEventRecord(s.ev, L->stream));
        }
        s.state = Loader::kCopying;
      } catch (const std::exception& ex) {
        fail_entry(e, ex.what(), &fire);
        --e.reads_in_flight;
        s = Loader::Slot{Loader::kFree, nullptr, 0, 0, 0, false, s.sig, s.ev};
      }
    }
    // ---- finished copies: the file's landed prefix grows; waiters whose partition is in are answered
    bool copying = false;
    for (int i = 0; i < C_slots; ++i) {
      Loader::Slot& s = L->slots[(size_t)i];
      if (s.state != Loader::kCopying) continue;
      bool done = false, bad = false;
      if (L->sdma) {
        const hsa_signal_value_t v = hsa_signal_load_scacquire(s.sig);
        done = v <= 0;
        bad = v < 0;
      } else {
        const hipError_t q = hipEventQuery(s.ev);
        done = q != hipErrorNotReady;
        bad = done && q != hipSuccess;
      }
      if (!done) {
        copying = true;
        continue;
      }
      std::shared_ptr<Entry> ep = s.e;
      Entry& e = *ep;
      --e.reads_in_flight;
      if (bad) {
        fail_entry(e, "H2D copy of " + e.path + " failed", &fire);
        if (L->sdma) SdmaEngine::arm(s.sig, 0);
      } else if (!e.failed) {
        e.done_chunks[s.off] = s.len;
        for (auto it = e.done_chunks.begin(); it != e.done_chunks.end() && it->first == e.landed;
             it = e.done_chunks.erase(it))
          e.landed += it->second;
        collect_ready(e, &fire);
        if (e.landed >= e.len) {
          e.loading = false;
          st_.loads++;
          st_.bytes_loaded += e.len;
          st_.load_ms += (now_s() - e.t_start) * 1000.0;
          st_.last_landed_boot_ms = boot_ms();
          collect_ready(e, &fire);
        }
      }
      if ((e.failed || !e.loading) && e.reads_in_flight == 0 && e.fd >= 0) {
        ::close(e.fd);
        e.fd = -1;
      }
      if (e.job_done && !e.loading && !e.failed) {  // JOB_OVER came while it was loading
        erase_entry(e.path);
        st_.evictions++;
      }
      s = Loader::Slot{Loader::kFree, nullptr, 0, 0, 0, false, s.sig, s.ev};
    }
    // ---- free slots: the next chunk of each file being loaded, in turn
    struct Submit {
      int slot, fd;
      int64_t off, len;
      bool direct;
    };
    std::vector<Submit> subs;
    for (int i = 0; i < C_slots && !L->active.empty(); ++i) {
      Loader::Slot& s = L->slots[(size_t)i];
      if (s.state != Loader::kFree) continue;
      std::shared_ptr<Entry> e;
      while (!L->active.empty() && !e) {
        e = L->active.front();
        L->active.pop_front();
        if (e->failed || e->next_read >= e->len) e.reset();
      }
      if (!e) break;
      const int64_t off = e->next_read, want = std::min(C, e->len - off);
      e->next_read += want;
      e->reads_in_flight++;
      if (e->next_read < e->len) L->active.push_back(e);
      s.state = Loader::kReading;
      s.e = e;
      s.off = off;
      s.len = want;
      s.read_done = false;
      s.result = 0;
      subs.push_back(Submit{i, e->fd, off, e->direct ? align_io(want) : want, e->direct});
    }
    const bool busy = !L->active.empty() || !subs.empty() || copying ||
                      std::any_of(L->slots.begin(), L->slots.end(), [](const Loader::Slot& s) { return s.state != 0; });
    if (busy != was_busy) {  // wall time with any loader busy
      if (busy && busy_loaders_++ == 0) busy_since_ = now_s();
      if (!busy && --busy_loaders_ == 0) st_.load_wall_ms += (now_s() - busy_since_) * 1000.0;
      was_busy = busy;
    }
    if (!subs.empty() && st_.first_read_boot_ms == 0) st_.first_read_boot_ms = boot_ms();
    if (!subs.empty() || !fire.empty()) {
      lk.unlock();
      // a chunk goes to disk as reads of opt_.read_bytes (the device sustains more small O_DIRECT reads in
      // flight than large ones); the chunk is landed when the last of them completes
      const int64_t R = opt_.read_bytes;
      for (const Submit& sb : subs) {
        Loader::Slot* sp = &L->slots[(size_t)sb.slot];
        {
          std::lock_guard<std::mutex> g(mu_);
          sp->parts = (int)((sb.len + R - 1) / R);
        }
        auto landed = [this, L, sp](int64_t r) {
          std::lock_guard<std::mutex> g(mu_);
          if (r < 0 || sp->result < 0)
            sp->result = -1;
          else
            sp->result += r;
          if (--sp->parts == 0) {
            sp->read_done = true;
            L->cv.notify_all();
          }
        };
        for (int64_t p = 0; p < sb.len; p += R) {
          uint8_t* dst = L->ring + (int64_t)sb.slot * C + p;
          const int64_t off = sb.off + p, n = std::min(R, sb.len - p);
          if (sb.direct) {
            L->aio->read(sb.fd, off, n, dst, landed);
            continue;
          }
          std::lock_guard<std::mutex> g(L->rmu);
          L->rq.push_back([fd = sb.fd, off, n, dst, landed] {
            int64_t got = 0;
            while (got < n) {
              const ssize_t r = ::pread(fd, dst + got, (size_t)(n - got), (off_t)(off + got));
              if (r < 0 && errno == EINTR) continue;
              if (r <= 0) break;
              got += r;
            }
            landed(got);
          });
          L->rcv.notify_one();
        }
      }
      for (Fire& f : fire) f.ready(f.ok, f.ref, f.why);
      fire.clear();
      lk.lock();
      continue;
    }
    if (L->stop && !busy && L->pending.empty() && L->opening == 0) break;
    if (copying)
      L->cv.wait_for(lk, std::chrono::microseconds(200));  // SDMA completions are polled
    else
      L->cv.wait_for(lk, std::chrono::milliseconds(50));
  }
  lk.unlock();
  if (L->aio) L->aio->drain();
  {
    std::lock_guard<std::mutex> g(L->rmu);  // queued reads still run: their slots' landing is awaited by nobody
    L->rstop = true;
    L->rcv.notify_all();
  }
  for (auto& t : L->readers) t.join();
  for (auto& s : L->slots) {
    if (L->sdma && s.sig.handle) L->sdma->destroy_signal(s.sig);
    if (s.ev) (void)hipEventDestroy(s.ev);
  }
  if (L->stream) (void)hipStreamDestroy(L->stream);
  if (L->ring) pinned_host_free(L->ring);
}

}  // namespace gpu
}  // namespace uda
