// Node-local shared-memory control plane. See uda/shm_group.h.
#include "uda/shm_group.h"

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace uda {

namespace {
constexpr uint64_t kMagic = 0x5544415348474d31ull;  // "UDASHGM1"
constexpr size_t kPage = 4096;

size_t page_up(size_t v) { return (v + kPage - 1) / kPage * kPage; }

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A crashed rank stays a zombie until its launcher reaps it: exited means gone or state Z/X.
bool process_alive(pid_t pid) {
  if (::kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return true;  // no procfs view: trust kill()
  char buf[512];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');  // comm may contain spaces
  if (!rp || rp[1] != ' ') return true;
  return rp[2] != 'Z' && rp[2] != 'X';
}

struct alignas(64) PaddedCtr {
  std::atomic<int64_t> v;
};
}  // namespace

struct ShmGroup::Header {
  std::atomic<uint64_t> magic;
  int32_t world;
  int32_t pad;
  uint64_t total;
  alignas(64) std::atomic<int32_t> attached;
  std::atomic<int32_t> aborted;  // 0 ok, 1 being written, 2 reason valid
  alignas(64) std::atomic<int64_t> bar_count;
  alignas(64) std::atomic<int64_t> bar_gen;
  char why[512];
};

struct ShmGroup::RankArea {
  alignas(64) std::atomic<int64_t> pid;  // 0 not attached, -1 left
  PaddedCtr ctr[kCounters];
  alignas(64) std::atomic<int32_t> nalloc;
  struct Alloc {
    uint8_t blob[kAllocBlob];
    int64_t size;
  } allocs[kMaxAllocs];
};

ShmGroup::Header* ShmGroup::hdr() const { return reinterpret_cast<Header*>(base_); }
ShmGroup::RankArea* ShmGroup::area(int r) const {
  return reinterpret_cast<RankArea*>(base_ + off_ranks_ + (size_t)r * page_up(sizeof(RankArea)));
}
uint8_t* ShmGroup::mailbox(int r) const { return base_ + off_mail_ + (size_t)r * page_up(mailbox_bytes_); }
uint8_t* ShmGroup::outbox(int r, int parity) const {
  return base_ + off_out_ + ((size_t)r * 2 + (size_t)(parity & 1)) * page_up(outbox_bytes_);
}

ShmGroup::ShmGroup(const std::string& name, int rank, int world, size_t mailbox_bytes, size_t outbox_bytes,
                   double timeout_s)
    : name_(name.empty() || name[0] != '/' ? "/" + name : name),
      rank_(rank),
      world_(world),
      mailbox_bytes_(std::max<size_t>(mailbox_bytes, 64 * (size_t)std::max(world, 1))),
      outbox_bytes_(std::max<size_t>(outbox_bytes, 64)),
      timeout_s_(timeout_s) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("ShmGroup: bad rank/world");
  if (name_.size() < 2 || name_.find('/', 1) != std::string::npos) throw std::runtime_error("ShmGroup: bad name");
  off_ranks_ = page_up(sizeof(Header));
  off_mail_ = off_ranks_ + (size_t)world * page_up(sizeof(RankArea));
  off_out_ = off_mail_ + (size_t)world * page_up(mailbox_bytes_);
  total_ = off_out_ + (size_t)world * 2 * page_up(outbox_bytes_);
  const double t0 = now_s();
  int fd = -1;
  if (rank == 0) {
    (void)shm_unlink(name_.c_str());  // a stale segment of a crashed run with the same name
    fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw std::runtime_error("ShmGroup: shm_open(" + name_ + ") failed: " + std::strerror(errno));
    if (ftruncate(fd, (off_t)total_) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name_.c_str());
      throw std::runtime_error("ShmGroup: ftruncate failed: " + std::string(std::strerror(e)));
    }
  } else {
    for (;;) {
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat sb;
        if (fstat(fd, &sb) == 0 && (size_t)sb.st_size == total_) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > timeout_s_) throw std::runtime_error("ShmGroup: segment " + name_ + " did not appear");
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  }
  void* p = mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("ShmGroup: mmap failed: " + std::string(std::strerror(errno)));
  base_ = static_cast<uint8_t*>(p);
  if (rank == 0) {
    hdr()->world = world;
    hdr()->total = total_;
    hdr()->magic.store(kMagic, std::memory_order_release);
  } else {
    while (hdr()->magic.load(std::memory_order_acquire) != kMagic) {
      if (now_s() - t0 > timeout_s_) {
        munmap(base_, total_);
        base_ = nullptr;
        throw std::runtime_error("ShmGroup: segment " + name_ + " never initialised");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (hdr()->world != world || hdr()->total != total_) {
      munmap(base_, total_);
      base_ = nullptr;
      throw std::runtime_error("ShmGroup: world/layout mismatch with the creator of " + name_);
    }
  }
  area(rank)->pid.store((int64_t)getpid(), std::memory_order_release);
  hdr()->attached.fetch_add(1, std::memory_order_acq_rel);
  try {
    barrier("attach");
  } catch (...) {
    if (rank == 0) (void)shm_unlink(name_.c_str());
    munmap(base_, total_);
    base_ = nullptr;
    throw;
  }
  if (rank == 0) (void)shm_unlink(name_.c_str());  // mappings keep the segment alive
}

ShmGroup::~ShmGroup() {
  if (!base_) return;
  area(rank_)->pid.store(-1, std::memory_order_release);
  munmap(base_, total_);
}

bool ShmGroup::aborted() const { return hdr()->aborted.load(std::memory_order_acquire) != 0; }

std::string ShmGroup::abort_reason() const {
  for (int i = 0; i < 1000 && hdr()->aborted.load(std::memory_order_acquire) == 1; ++i)
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  if (hdr()->aborted.load(std::memory_order_acquire) != 2) return "unknown";
  return std::string(hdr()->why, strnlen(hdr()->why, sizeof(hdr()->why)));
}

void ShmGroup::abort(const std::string& why) {
  int32_t expect = 0;
  if (!hdr()->aborted.compare_exchange_strong(expect, 1, std::memory_order_acq_rel)) return;
  const std::string msg = "rank " + std::to_string(rank_) + ": " + why;
  std::strncpy(hdr()->why, msg.c_str(), sizeof(hdr()->why) - 1);
  hdr()->why[sizeof(hdr()->why) - 1] = 0;
  hdr()->aborted.store(2, std::memory_order_release);
}

void ShmGroup::check() const {
  if (aborted()) throw std::runtime_error("rank group aborted: " + abort_reason());
}

void ShmGroup::check_peers_alive() {
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    const int64_t pid = area(r)->pid.load(std::memory_order_acquire);
    if (pid == -1) abort("rank " + std::to_string(r) + " left the group while a peer waited for it");
    if (pid > 0 && !process_alive((pid_t)pid))
      abort("rank " + std::to_string(r) + " (pid " + std::to_string(pid) + ") died");
  }
}

template <typename Pred>
void ShmGroup::spin_wait(Pred ready, const char* what, double timeout_s, bool abort_on_timeout) {
  const double t0 = now_s();
  double last_check = t0;
  for (int spin = 0; !ready(); ++spin) {
    if (aborted())
      throw std::runtime_error(std::string("rank group aborted while waiting for ") + what + ": " + abort_reason());
    if (spin < 128) {
      __builtin_ia32_pause();
    } else if (spin < 1024) {
      sched_yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(spin < 4096 ? 10 : 50));
    }
    if ((spin & 63) == 63) {
      const double t = now_s();
      if (t - last_check > 0.05) {
        last_check = t;
        check_peers_alive();
      }
      if (t - t0 > timeout_s) {
        const std::string msg = std::string("timed out after ") + std::to_string((int)timeout_s) + " s waiting for " + what;
        if (abort_on_timeout) abort(msg);
        throw std::runtime_error(msg);
      }
    }
  }
}

void ShmGroup::barrier(const char* what) {
  Header* h = hdr();
  const int64_t gen = h->bar_gen.load(std::memory_order_acquire);
  if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == world_) {
    h->bar_count.store(0, std::memory_order_relaxed);
    h->bar_gen.fetch_add(1, std::memory_order_acq_rel);
    return;
  }
  spin_wait([&] { return h->bar_gen.load(std::memory_order_acquire) != gen; }, what, timeout_s_, true);
}

bool ShmGroup::try_barrier(double timeout_s) {
  Header* h = hdr();
  const int64_t gen = h->bar_gen.load(std::memory_order_acquire);
  if (h->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == world_) {
    h->bar_count.store(0, std::memory_order_relaxed);
    h->bar_gen.fetch_add(1, std::memory_order_acq_rel);
    return true;
  }
  try {
    spin_wait([&] { return h->bar_gen.load(std::memory_order_acquire) != gen; }, "teardown barrier", timeout_s, false);
    return true;
  } catch (...) {
    return false;
  }
}

void ShmGroup::publish(Counter c, int64_t v) { area(rank_)->ctr[c].v.store(v, std::memory_order_release); }

int64_t ShmGroup::read(Counter c, int peer) const { return area(peer)->ctr[c].v.load(std::memory_order_acquire); }

void ShmGroup::wait_at_least(Counter c, int peer, int64_t v, const char* what) {
  if (peer >= 0) {
    spin_wait([&] { return read(c, peer) >= v; }, what, timeout_s_, true);
    return;
  }
  spin_wait(
      [&] {
        for (int r = 0; r < world_; ++r)
          if (r != rank_ && read(c, r) < v) return false;
        return true;
      },
      what, timeout_s_, true);
}

void ShmGroup::alltoall_i64(const int64_t* send, int64_t* recv, size_t n) {
  const size_t per = mailbox_bytes_ / 8 / (size_t)world_;  // int64 per peer per chunk
  for (size_t b = 0; b < n || (n == 0 && b == 0); b += per) {
    const size_t k = std::min(per, n - b);
    int64_t* mine = reinterpret_cast<int64_t*>(mailbox(rank_));
    for (int p = 0; p < world_; ++p) std::memcpy(mine + (size_t)p * per, send + (size_t)p * n + b, k * 8);
    barrier("alltoall (write)");
    for (int p = 0; p < world_; ++p)
      std::memcpy(recv + (size_t)p * n + b, reinterpret_cast<int64_t*>(mailbox(p)) + (size_t)rank_ * per, k * 8);
    barrier("alltoall (read)");
    if (n == 0) break;
  }
}

int ShmGroup::publish_alloc(const void* blob, size_t len, int64_t size) {
  if (len > (size_t)kAllocBlob) throw std::runtime_error("ShmGroup: allocation blob too large");
  RankArea* a = area(rank_);
  const int id = a->nalloc.load(std::memory_order_relaxed);
  if (id >= kMaxAllocs) throw std::runtime_error("ShmGroup: too many exported allocations");
  std::memset(a->allocs[id].blob, 0, kAllocBlob);
  std::memcpy(a->allocs[id].blob, blob, len);
  a->allocs[id].size = size;
  a->nalloc.store(id + 1, std::memory_order_release);
  return id;
}

bool ShmGroup::read_alloc(int peer, int id, void* blob, size_t len, int64_t* size) const {
  RankArea* a = area(peer);
  if (id < 0 || id >= a->nalloc.load(std::memory_order_acquire)) return false;
  std::memcpy(blob, a->allocs[id].blob, std::min(len, (size_t)kAllocBlob));
  if (size) *size = a->allocs[id].size;
  return true;
}

}  // namespace uda
