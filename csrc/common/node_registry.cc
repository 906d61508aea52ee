// Node-local registry of reduce tasks and HBM bytes per GPU. See uda/node_registry.h.
#include "uda/node_registry.h"

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace uda {

namespace {
constexpr uint64_t kMagic = 0x55444e4f44455231ull;  // "UDANODER1"
constexpr int32_t kVersion = 1;
enum Kind : int32_t { kFree = 0, kTask = 1, kBytes = 2 };

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

uint64_t process_start_ticks(int pid) {
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');  // comm may hold spaces and parentheses
  if (!p) return 0;
  // after ") ": field 3 (state) ... field 22 (starttime)
  int field = 2;
  for (++p; *p && field < 22; ++p)
    if (*p == ' ') ++field;
  return field == 22 ? std::strtoull(p, nullptr, 10) : 0;
}

bool process_running(int pid, uint64_t start) {
  if (pid <= 0) return false;
  if (::kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return true;  // no procfs view: trust kill()
  char buf[1024];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');
  if (!rp || rp[1] != ' ') return true;
  if (rp[2] == 'Z' || rp[2] == 'X') return false;  // exited, not yet reaped
  return start == 0 || process_start_ticks(pid) == start;
}

struct NodeRegistry::Header {
  std::atomic<uint64_t> magic;
  int32_t version;
  int32_t ndev;
  uint64_t total;
  pthread_mutex_t mu;
  char keys[kMaxDevices][kKeyBytes];
};

struct NodeRegistry::Slot {
  int32_t kind;
  int32_t pid;
  uint64_t start;
  int32_t dev;
  int32_t pad;
  int64_t bytes;
  int64_t resident;
  char tag[kTagBytes];
};

// Robust process-shared mutex: a holder that died leaves EOWNERDEAD, and the table it guarded holds
// only whole-field stores, so the next owner marks it consistent and goes on.
struct NodeRegistry::Lock {
  pthread_mutex_t* m;
  explicit Lock(pthread_mutex_t* mu) : m(mu) {
    const int r = pthread_mutex_lock(m);
    if (r == EOWNERDEAD) {
      pthread_mutex_consistent(m);
    } else if (r != 0) {
      throw std::runtime_error("node registry: lock failed: " + std::string(std::strerror(r)));
    }
  }
  ~Lock() { pthread_mutex_unlock(m); }
};

NodeRegistry::Header* NodeRegistry::hdr() const { return reinterpret_cast<Header*>(base_); }
NodeRegistry::Slot* NodeRegistry::slots() const {
  return reinterpret_cast<Slot*>(base_ + ((sizeof(Header) + 63) & ~(size_t)63));
}

NodeRegistry::NodeRegistry(const std::string& name) {
  if (!name.empty()) {
    name_ = name[0] == '/' ? name : "/" + name;
  } else if (const char* e = std::getenv("UDA_NODE_REGISTRY"); e && *e) {
    name_ = e[0] == '/' ? e : std::string("/") + e;
  } else {
    name_ = "/uda_node_v1." + std::to_string((long)getuid());
  }
  if (name_.size() < 2 || name_.find('/', 1) != std::string::npos) throw std::runtime_error("node registry: bad name " + name_);
  total_ = ((sizeof(Header) + 63) & ~(size_t)63) + sizeof(Slot) * kMaxSlots;
  pid_ = (int)getpid();
  start_ = process_start_ticks(pid_);
  for (int attempt = 0; attempt < 2; ++attempt) {
    int fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    const bool creator = fd >= 0;
    if (!creator) {
      if (errno != EEXIST) throw std::runtime_error("node registry: shm_open(" + name_ + "): " + std::strerror(errno));
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd < 0) {
        if (errno == ENOENT) continue;  // unlinked between the two calls
        throw std::runtime_error("node registry: shm_open(" + name_ + "): " + std::strerror(errno));
      }
    } else if (ftruncate(fd, (off_t)total_) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name_.c_str());
      throw std::runtime_error("node registry: ftruncate: " + std::string(std::strerror(e)));
    }
    // an opener may see the segment before its creator sized and initialized it
    const double t0 = now_s();
    bool ready = creator;
    while (!ready) {
      struct stat sb;
      if (fstat(fd, &sb) == 0 && (size_t)sb.st_size >= total_) {
        void* p = mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (p != MAP_FAILED) {
          auto* h = static_cast<Header*>(p);
          if (h->magic.load(std::memory_order_acquire) == kMagic) {
            if (h->version != kVersion || h->total != total_) {
              munmap(p, total_);
              close(fd);
              throw std::runtime_error("node registry: " + name_ + " has another layout");
            }
            base_ = static_cast<uint8_t*>(p);
            ready = true;
            break;
          }
          munmap(p, total_);
        }
      }
      if (now_s() - t0 > 2.0) break;  // its creator died before initializing it
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (!ready) {
      close(fd);
      shm_unlink(name_.c_str());
      continue;
    }
    if (creator) {
      void* p = mmap(nullptr, total_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p == MAP_FAILED) {
        const int e = errno;
        close(fd);
        shm_unlink(name_.c_str());
        throw std::runtime_error("node registry: mmap: " + std::string(std::strerror(e)));
      }
      base_ = static_cast<uint8_t*>(p);
      std::memset(base_, 0, total_);
      Header* h = hdr();
      h->version = kVersion;
      h->total = total_;
      pthread_mutexattr_t a;
      pthread_mutexattr_init(&a);
      pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
      pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
      pthread_mutex_init(&h->mu, &a);
      pthread_mutexattr_destroy(&a);
      h->magic.store(kMagic, std::memory_order_release);
    }
    close(fd);
    return;
  }
  throw std::runtime_error("node registry: cannot open " + name_);
}

NodeRegistry::~NodeRegistry() {
  if (!base_) return;
  try {
    Lock l(&hdr()->mu);
    for (int i = 0; i < kMaxSlots; ++i) {
      Slot& s = slots()[i];
      if (s.kind != kFree && s.pid == pid_ && s.start == start_) s.kind = kFree;
    }
  } catch (...) {
  }
  munmap(base_, total_);
}

NodeRegistry* NodeRegistry::instance() {
  static NodeRegistry* r = [] () -> NodeRegistry* {
    try {
      return new NodeRegistry();  // never destroyed: its slots die with the process (reaped by pid)
    } catch (const std::exception& e) {
      std::fprintf(stderr, "[uda] node registry unavailable: %s\n", e.what());
      return nullptr;
    }
  }();
  return r;
}

void NodeRegistry::unlink() { shm_unlink(name_.c_str()); }

int NodeRegistry::device_index(const std::string& key, bool create) {
  Header* h = hdr();
  std::string k = key.substr(0, kKeyBytes - 1);
  for (int i = 0; i < h->ndev; ++i)
    if (k == h->keys[i]) return i;
  if (!create) return -1;
  if (h->ndev >= kMaxDevices) throw std::runtime_error("node registry: more than 64 devices");
  std::snprintf(h->keys[h->ndev], kKeyBytes, "%s", k.c_str());
  return h->ndev++;
}

void NodeRegistry::reap() {
  std::map<std::pair<int, uint64_t>, bool> alive;  // one /proc look per process
  for (int i = 0; i < kMaxSlots; ++i) {
    Slot& s = slots()[i];
    if (s.kind == kFree) continue;
    if (s.pid == pid_ && s.start == start_) continue;
    auto key = std::make_pair((int)s.pid, s.start);
    auto it = alive.find(key);
    if (it == alive.end()) it = alive.emplace(key, process_running(s.pid, s.start)).first;
    if (!it->second) {
      s.kind = kFree;
      ++reclaimed_;
    }
  }
}

int NodeRegistry::take_slot() {
  for (int i = 0; i < kMaxSlots; ++i)
    if (slots()[i].kind == kFree) return i;
  throw std::runtime_error("node registry: no free slot");
}

NodeRegistry::Placement NodeRegistry::place_task(const std::vector<std::string>& keys, const std::string& tag) {
  Placement pl;
  if (keys.empty()) return pl;
  Lock l(&hdr()->mu);
  reap();
  std::vector<int> di(keys.size());
  std::vector<int> tasks(keys.size(), 0);
  std::vector<int64_t> bytes(keys.size(), 0);
  for (size_t k = 0; k < keys.size(); ++k) di[k] = device_index(keys[k], true);
  for (int i = 0; i < kMaxSlots; ++i) {
    const Slot& s = slots()[i];
    if (s.kind == kFree) continue;
    for (size_t k = 0; k < keys.size(); ++k)
      if (s.dev == di[k]) {
        if (s.kind == kTask) ++tasks[k];
        if (s.kind == kBytes) bytes[k] += s.bytes;
      }
  }
  size_t best = 0;
  for (size_t k = 1; k < keys.size(); ++k)
    if (tasks[k] < tasks[best] || (tasks[k] == tasks[best] && bytes[k] < bytes[best])) best = k;
  const int i = take_slot();
  Slot& s = slots()[i];
  s.pid = pid_;
  s.start = start_;
  s.dev = di[best];
  s.bytes = s.resident = 0;
  std::snprintf(s.tag, kTagBytes, "%s", tag.c_str());
  s.kind = kTask;
  pl.index = (int)best;
  pl.slot = i;
  return pl;
}

int NodeRegistry::add_task(const std::string& key, const std::string& tag) {
  Lock l(&hdr()->mu);
  const int d = device_index(key, true);
  const int i = take_slot();
  Slot& s = slots()[i];
  s.pid = pid_;
  s.start = start_;
  s.dev = d;
  s.bytes = s.resident = 0;
  std::snprintf(s.tag, kTagBytes, "%s", tag.c_str());
  s.kind = kTask;
  return i;
}

void NodeRegistry::release(int slot) {
  if (slot < 0 || slot >= kMaxSlots) return;
  Lock l(&hdr()->mu);
  Slot& s = slots()[slot];
  if (s.kind == kTask && s.pid == pid_ && s.start == start_) s.kind = kFree;
}

void NodeRegistry::set_bytes(const std::string& key, int64_t bytes, int64_t resident) {
  Lock l(&hdr()->mu);
  const int d = device_index(key, true);
  auto mine = [&](const Slot& s) { return s.kind == kBytes && s.pid == pid_ && s.start == start_ && s.dev == d; };
  if ((int)my_bytes_slot_.size() <= d) my_bytes_slot_.resize((size_t)d + 1, -1);
  int at = my_bytes_slot_[(size_t)d];
  if (at < 0 || !mine(slots()[at])) {
    at = -1;
    for (int i = 0; i < kMaxSlots && at < 0; ++i)
      if (mine(slots()[i])) at = i;
  }
  if (at < 0) {
    if (bytes == 0 && resident == 0) return;
    for (int i = 0; i < kMaxSlots && at < 0; ++i)
      if (slots()[i].kind == kFree) at = i;
    if (at < 0) {
      reap();
      at = take_slot();
    }
    Slot& s = slots()[at];
    s.pid = pid_;
    s.start = start_;
    s.dev = d;
    std::snprintf(s.tag, kTagBytes, "hbm");
    s.kind = kBytes;
  }
  slots()[at].bytes = bytes;
  slots()[at].resident = resident;
  my_bytes_slot_[(size_t)d] = at;
}

NodeRegistry::Use NodeRegistry::usage(const std::string& key) {
  Use u;
  Lock l(&hdr()->mu);
  // the byte budget asks often (every allocation): look for dead processes at most every 100 ms
  if (now_s() - last_reap_ > 0.1) {
    reap();
    last_reap_ = now_s();
  }
  const int d = device_index(key, false);
  if (d < 0) return u;
  for (int i = 0; i < kMaxSlots; ++i) {
    const Slot& s = slots()[i];
    if (s.kind == kFree || s.dev != d) continue;
    if (s.kind == kTask) ++u.tasks;
    if (s.kind == kBytes) {
      u.bytes += s.bytes;
      u.resident += s.resident;
    }
  }
  return u;
}

}  // namespace uda
