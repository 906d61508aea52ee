// Explicit SDMA delivery copies and NUMA-local pinned memory. See sdma.h.
#include "sdma.h"
#include "uda/topology.h"

#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <mutex>
#include <thread>
#include <atomic>
#include <map>
#include <unordered_map>
#include <vector>

#include "uda/log.h"

namespace uda {
namespace gpu {

namespace {
void hsa_check(hsa_status_t s, const char* what) {
  if (s != HSA_STATUS_SUCCESS) {
    const char* msg = nullptr;
    hsa_status_string(s, &msg);
    throw std::runtime_error(std::string("HSA error in ") + what + ": " + (msg ? msg : "?"));
  }
}

struct PciAddr {
  unsigned domain = 0, bus = 0, dev = 0, func = 0;
  bool ok = false;
};

PciAddr hip_pci(int device) {
  PciAddr a;
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), device) != hipSuccess) return a;
  if (std::sscanf(buf, "%x:%x:%x.%x", &a.domain, &a.bus, &a.dev, &a.func) == 4) a.ok = true;
  return a;
}

struct AgentScan {
  PciAddr want;
  std::vector<hsa_agent_t> gpus, cpus;
  hsa_agent_t match{};
  bool found = false;
};

hsa_status_t scan_agent(hsa_agent_t agent, void* data) {
  auto* sc = static_cast<AgentScan*>(data);
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (type == HSA_DEVICE_TYPE_CPU) {
    sc->cpus.push_back(agent);
  } else if (type == HSA_DEVICE_TYPE_GPU) {
    sc->gpus.push_back(agent);
    uint32_t bdf = 0, domain = 0;
    if (sc->want.ok &&
        hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS) {
      (void)hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain);
      const uint32_t want = (sc->want.bus << 8) | (sc->want.dev << 3) | sc->want.func;
      if (bdf == want && domain == sc->want.domain && !sc->found) {
        sc->match = agent;
        sc->found = true;
      }
    }
  }
  return HSA_STATUS_SUCCESS;
}

struct PoolScan {
  hsa_amd_memory_pool_t coarse{}, fine{};
  bool has_coarse = false, has_fine = false;
};

hsa_status_t scan_pool(hsa_amd_memory_pool_t pool, void* data) {
  auto* ps = static_cast<PoolScan*>(data);
  hsa_amd_segment_t seg;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  bool alloc_ok = false;
  (void)hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
  if (!alloc_ok) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  (void)hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !ps->has_coarse) {
    ps->coarse = pool;
    ps->has_coarse = true;
  } else if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) &&
             !(flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !ps->has_fine) {
    ps->fine = pool;
    ps->has_fine = true;
  }
  return HSA_STATUS_SUCCESS;
}

std::string read_line(const std::string& path) {
  std::ifstream f(path);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}
}  // namespace

int device_numa_node(int device) {
  const PciAddr a = hip_pci(device);
  if (!a.ok) return -1;
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%04x:%02x:%02x.%x/numa_node", a.domain, a.bus, a.dev,
                a.func);
  const std::string s = read_line(path);
  if (s.empty()) return -1;
  return std::atoi(s.c_str());
}

std::vector<int> device_consumer_cpus(int device) {
  // the process's CPUs as it started (threads bound later must not narrow the slice of the next one)
  static const std::vector<int> allowed = allowed_cpus();
  const PciAddr a = hip_pci(device);
  if (!a.ok) return {};
  GpuLocation me;
  me.domain = a.domain;
  me.bus = a.bus;
  me.dev = a.dev;
  me.func = a.func;
  me.numa_node = pci_numa_node(a.domain, a.bus, a.dev, a.func);
  const char* e = std::getenv("UDA_CONSUMER_CPUS");
  if (e && std::string(e) == "node") return consumer_cpus(me, {me}, allowed);
  // the GPUs this process can use share their nodes' CPUs (a one-GPU container on an 8-GPU host keeps
  // its whole NUMA node; the eight ranks of an 8-GPU job get disjoint slices)
  static const std::vector<GpuLocation> gpus = usable_gpus();
  return consumer_cpus(me, gpus, allowed);
}

void bind_thread_to_numa(int node) {
  if (node < 0) return;
  const std::string list = read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  if (list.empty()) return;
  cpu_set_t allowed, want;
  CPU_ZERO(&want);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  std::stringstream ss(list);
  std::string tok;
  int n = 0;
  while (std::getline(ss, tok, ',')) {
    int lo = 0, hi = 0;
    if (std::sscanf(tok.c_str(), "%d-%d", &lo, &hi) != 2) hi = lo = std::atoi(tok.c_str());
    for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) {
        CPU_SET(c, &want);
        ++n;
      }
  }
  if (n > 0) (void)sched_setaffinity(0, sizeof(want), &want);
}

namespace {
std::mutex g_pin_mu;
std::unordered_map<void*, std::pair<void*, size_t>>& pinned_maps() {  // aligned ptr -> (mapping, length)
  static auto* m = new std::unordered_map<void*, std::pair<void*, size_t>>();
  return *m;
}

void* hip_host_malloc_on_node(size_t bytes, int node) {
  void* p = nullptr;
  if (node < 0 || node >= 64) {
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) throw std::runtime_error("hipHostMalloc failed");
    return p;
  }
  const unsigned long mask = 1ul << node;
  constexpr int kMpolDefault = 0, kMpolPreferred = 1;
  const bool policy = syscall(SYS_set_mempolicy, kMpolPreferred, &mask, sizeof(mask) * 8) == 0;
  const hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault | hipHostMallocNumaUser);
  if (policy) (void)syscall(SYS_set_mempolicy, kMpolDefault, nullptr, 0);
  if (e != hipSuccess) throw std::runtime_error("hipHostMalloc (NUMA node " + std::to_string(node) + ") failed");
  return p;
}

struct SharedRegion {
  size_t len;
  int fd;
  uint64_t id;
  int node;  // NUMA node the pages were bound to (-1: any)
};
std::atomic<bool> g_shareable{false};
std::atomic<uint64_t> g_next_share_id{1};
std::map<uintptr_t, SharedRegion>& shared_regions() {  // aligned start -> region (under g_pin_mu)
  static auto* m = new std::map<uintptr_t, SharedRegion>();
  return *m;
}

// mmap + hugepage advice + parallel first touch + hipHostRegister; nullptr if any step fails. In
// shareable mode the pages are a memfd mapped shared at the aligned start (the rest of the
// reservation stays an inaccessible anonymous mapping).
void* register_fresh_pages(size_t bytes, int node) {
  constexpr size_t kHuge = (size_t)2 << 20;
  const size_t len = (bytes + kHuge - 1) & ~(kHuge - 1);
  const size_t maplen = len + kHuge;  // room to align the start to a huge page
  const bool share = g_shareable.load();
  void* m = mmap(nullptr, maplen, share ? PROT_NONE : PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return nullptr;
  uint8_t* a = reinterpret_cast<uint8_t*>(((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
  int fd = -1;
  if (share) {
    fd = (int)syscall(SYS_memfd_create, "uda-pinned", 1u /* MFD_CLOEXEC */);
    if (fd < 0 || ftruncate(fd, (off_t)len) != 0 ||
        mmap(a, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED, fd, 0) == MAP_FAILED) {
      if (fd >= 0) close(fd);
      munmap(m, maplen);
      return nullptr;
    }
  }
  (void)madvise(a, len, MADV_HUGEPAGE);
  (void)madvise(m, maplen, MADV_DONTFORK);  // a forked child must not copy (or share) pinned pages
  if (node >= 0 && node < 64) {
    const unsigned long mask = 1ul << node;
    constexpr int kMpolPreferred = 1;
    (void)syscall(SYS_mbind, a, len, kMpolPreferred, &mask, sizeof(mask) * 8, 0);
  }
  // first touch: the kernel zeroes the pages in the touching threads, not inside the registration
  const int nt = (int)std::max<size_t>(1, std::min<size_t>(8, len / ((size_t)32 << 20)));
  const size_t per = (len / nt + kHuge - 1) & ~(kHuge - 1);
  std::vector<std::thread> ts;
  for (int t = 0; t < nt; ++t)
    ts.emplace_back([=] {
      const size_t b = (size_t)t * per;
      if (b >= len) return;
      const size_t n = std::min(per, len - b);
      for (size_t o = 0; o < n; o += 4096) a[b + o] = 0;
    });
  for (auto& t : ts) t.join();
  auto undo = [&] {
    if (fd >= 0) close(fd);
    munmap(m, maplen);
    return nullptr;
  };
  if (hipHostRegister(a, len, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    return undo();
  }
  void* d = nullptr;  // copies and kernels use the host address: it must be the device address too
  if (hipHostGetDevicePointer(&d, a, 0) != hipSuccess || d != a) {
    (void)hipGetLastError();
    (void)hipHostUnregister(a);
    return undo();
  }
  std::lock_guard<std::mutex> g(g_pin_mu);
  pinned_maps()[a] = {m, maplen};
  if (fd >= 0)
    shared_regions()[(uintptr_t)a] = SharedRegion{len, fd, g_next_share_id.fetch_add(1), node >= 0 && node < 64 ? node : -1};
  return a;
}
}  // namespace

void* pinned_host_alloc(size_t bytes, int node) {
  static const bool reg = [] {
    const char* e = std::getenv("UDA_PINNED_REGISTER");
    return !e || std::atoi(e) != 0;
  }();
  if (bytes == 0) bytes = 1;
  if (reg)
    if (void* p = register_fresh_pages(bytes, node)) return p;
  return hip_host_malloc_on_node(bytes, node);
}

void pinned_host_free(void* p) {
  if (!p) return;
  std::pair<void*, size_t> m{nullptr, 0};
  {
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = pinned_maps().find(p);
    if (it != pinned_maps().end()) {
      m = it->second;
      pinned_maps().erase(it);
    }
    auto sr = shared_regions().find((uintptr_t)p);
    if (sr != shared_regions().end()) {
      close(sr->second.fd);  // clients keep their own mappings of the pages until they unmap
      shared_regions().erase(sr);
    }
  }
  if (m.first) {
    (void)hipHostUnregister(p);
    munmap(m.first, m.second);
  } else {
    (void)hipHostFree(p);
  }
}

void* hip_host_alloc_on_node(size_t bytes, int node) { return pinned_host_alloc(bytes, node); }

void set_pinned_shareable(bool on) { g_shareable.store(on); }

bool pinned_share_of(const void* p, size_t len, PinnedShare* out) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> g(g_pin_mu);
  auto& m = shared_regions();
  auto it = m.upper_bound(a);
  if (it == m.begin()) return false;
  --it;
  if (a + len > it->first + it->second.len) return false;
  out->fd = it->second.fd;
  out->id = it->second.id;
  out->offset = a - it->first;
  out->region_bytes = it->second.len;
  out->numa_node = it->second.node;
  return true;
}

std::string numa_residency(const void* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::ifstream maps("/proc/self/maps");
  std::string line;
  uintptr_t start = 0;
  bool found = false;
  while (std::getline(maps, line)) {
    unsigned long lo = 0, hi = 0;
    if (std::sscanf(line.c_str(), "%lx-%lx", &lo, &hi) == 2 && a >= lo && a < hi) {
      start = lo;
      found = true;
      break;
    }
  }
  if (!found) return "unknown";
  std::ifstream nm("/proc/self/numa_maps");
  while (std::getline(nm, line)) {
    unsigned long lo = 0;
    if (std::sscanf(line.c_str(), "%lx", &lo) != 1 || lo != start) continue;
    std::stringstream ss(line);
    std::string tok;
    std::vector<std::pair<int, long>> nodes;
    long total = 0;
    while (ss >> tok) {
      int n = 0;
      long c = 0;
      if (std::sscanf(tok.c_str(), "N%d=%ld", &n, &c) == 2) {
        nodes.push_back({n, c});
        total += c;
      }
    }
    if (total == 0) return "untouched";
    std::string out;
    for (auto& nc : nodes) {
      if (!out.empty()) out += ",";
      out += "N" + std::to_string(nc.first) + "=" + std::to_string((nc.second * 100 + total / 2) / total) + "%";
    }
    return out;
  }
  return "unknown";
}

SdmaEngine::SdmaEngine(int device) {
  hsa_check(hsa_init(), "hsa_init");  // reference counted: HIP already initialised the runtime
  hsa_inited_ = true;
  AgentScan sc;
  sc.want = hip_pci(device);
  hsa_check(hsa_iterate_agents(scan_agent, &sc), "hsa_iterate_agents");
  if (!sc.found) {
    if (sc.gpus.size() == 1) {
      sc.match = sc.gpus[0];
    } else {
      throw std::runtime_error("SdmaEngine: no HSA GPU agent matches HIP device " + std::to_string(device));
    }
  }
  gpu_ = sc.match;
  if (sc.cpus.empty()) throw std::runtime_error("SdmaEngine: no HSA CPU agent");
  hsa_agent_t near{};
  if (hsa_agent_get_info(gpu_, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &near) == HSA_STATUS_SUCCESS &&
      near.handle != 0)
    cpu_ = near;
  else
    cpu_ = sc.cpus[0];
  PoolScan ps;
  hsa_check(hsa_amd_agent_iterate_memory_pools(cpu_, scan_pool, &ps), "iterate host pools");
  if (ps.has_coarse)
    host_pool_ = ps.coarse;
  else if (ps.has_fine)
    host_pool_ = ps.fine;
  else
    throw std::runtime_error("SdmaEngine: no allocatable host memory pool on the nearest CPU agent");
  numa_node_ = device_numa_node(device);
  uint32_t mask = 0, pref = 0;
  if (hsa_amd_memory_copy_engine_status(cpu_, gpu_, &mask) != HSA_STATUS_SUCCESS) mask = 0;
  if (hsa_amd_memory_get_preferred_copy_engine(cpu_, gpu_, &pref) != HSA_STATUS_SUCCESS) pref = 0;
  // One engine: on MI355X a single SDMA engine streams device -> host at the PCIe roof
  // (55.5-55.7 GB/s for engines 0, 1 or 2), two engines at once contend (47-50 GB/s) and engines 4-7
  // reach only 25 GB/s (profiles/r2_sdma_engine_sweep.md). Prefer the runtime's recommendation.
  uint32_t use = (pref & mask) ? (pref & mask) : mask;
  use &= (~use + 1u);  // lowest set bit
  if (const char* e = std::getenv("UDA_SDMA_ENGINE_MASK")) {  // operator override / sweeps
    const uint32_t want = (uint32_t)std::strtoul(e, nullptr, 0);
    if (want & mask) use = want & mask;
  }
  for (int b = 0; b < 16; ++b)
    if (use & (1u << b)) engine_ids_.push_back(1u << b);
  uint32_t hmask = 0;
  if (hsa_amd_memory_copy_engine_status(gpu_, cpu_, &hmask) != HSA_STATUS_SUCCESS) hmask = 0;
  uint32_t other = hmask & ~use;  // staging on a different engine than delivery
  if (other & 0xFu) other &= 0xFu;  // engines 4-7 stream at half the rate (r2_sdma_engine_sweep.md)
  const uint32_t pick = other ? other : hmask;
  h2d_engine_ = pick & (~pick + 1u);
  // Several processes staging on one GPU (rank processes sharing a device, or the store loader next to a
  // staging task) each get their own SDMA queue; on one engine those queues take turns. Spread them:
  // the process's local rank (or its pid) picks among the candidate engines. UDA_SDMA_H2D_SPREAD=0 keeps
  // every process on the lowest one.
  const char* spread = std::getenv("UDA_SDMA_H2D_SPREAD");
  if (!(spread && std::atoi(spread) == 0)) {
    std::vector<uint32_t> cand;
    for (int b = 0; b < 16; ++b)
      if (pick & (1u << b)) cand.push_back(1u << b);
    const char* lr = std::getenv("LOCAL_RANK");
    const int who = lr ? std::atoi(lr) : (int)getpid();
    if (cand.size() > 1) h2d_engine_ = cand[(size_t)who % cand.size()];
  }
  UDA_LOG(kInfo, "SDMA delivery: device %d numa %d engines mask 0x%x preferred 0x%x", device, numa_node_, mask, pref);
}

void SdmaEngine::warm(void* dev_scratch) {
  void* host = pinned_host_alloc(4096);
  hsa_signal_t sig = make_signal();
  try {
    arm(sig, 1);
    copy_h2d(dev_scratch, host, 4096, sig);
    wait(sig);
    arm(sig, parts(4096, 1));
    copy_d2h(host, dev_scratch, 4096, sig, 1);
    wait(sig);
  } catch (...) {
    destroy_signal(sig);
    pinned_host_free(host);
    throw;
  }
  destroy_signal(sig);
  pinned_host_free(host);
}

SdmaEngine::~SdmaEngine() {
  if (hsa_inited_) (void)hsa_shut_down();
}

SdmaEngine& SdmaEngine::for_device(int device) {
  static std::mutex mu;
  static std::map<int, SdmaEngine*>* engines = new std::map<int, SdmaEngine*>();  // leaked on purpose
  std::lock_guard<std::mutex> g(mu);
  auto it = engines->find(device);
  if (it == engines->end()) it = engines->emplace(device, new SdmaEngine(device)).first;
  return *it->second;
}

void* SdmaEngine::acquire_ring(size_t bytes) {
  {
    std::lock_guard<std::mutex> g(ring_mu_);
    auto it = ring_cache_.find(bytes);
    if (it != ring_cache_.end()) {
      void* p = it->second;
      ring_cache_.erase(it);
      return p;
    }
  }
  return alloc_host(bytes);
}

void SdmaEngine::release_ring(void* p, size_t bytes) {
  if (!p) return;
  std::lock_guard<std::mutex> g(ring_mu_);
  ring_cache_.emplace(bytes, p);
}

void* SdmaEngine::alloc_host(size_t bytes) {
  void* p = nullptr;
  if (g_shareable.load()) {
    // merge service: delivery rings its clients map (memfd-backed, registered; sdma.h)
    try {
      p = pinned_host_alloc(bytes, numa_node_);
      PinnedShare ps;
      if (pinned_share_of(p, 1, &ps)) return p;
      pinned_host_free(p);  // registration of the shared pages failed: the host pool, not shareable
    } catch (const std::exception&) {
    }
    p = nullptr;
  }
  hsa_check(hsa_amd_memory_pool_allocate(host_pool_, bytes, 0, &p), "host pool allocate");
  hsa_status_t s = hsa_amd_agents_allow_access(1, &gpu_, nullptr, p);
  if (s != HSA_STATUS_SUCCESS) {
    (void)hsa_amd_memory_pool_free(p);
    hsa_check(s, "agents_allow_access");
  }
  return p;
}

void SdmaEngine::free_host(void* p) {
  if (!p) return;
  PinnedShare ps;
  if (pinned_share_of(p, 1, &ps))
    pinned_host_free(p);
  else
    (void)hsa_amd_memory_pool_free(p);
}

hsa_signal_t SdmaEngine::make_signal() {
  hsa_signal_t s;
  hsa_check(hsa_signal_create(0, 0, nullptr, &s), "signal_create");
  return s;
}

void SdmaEngine::destroy_signal(hsa_signal_t s) {
  if (s.handle) (void)hsa_signal_destroy(s);
}

void SdmaEngine::arm(hsa_signal_t s, int64_t parts) { hsa_signal_store_screlease(s, parts); }
void SdmaEngine::add(hsa_signal_t s, int64_t parts) { hsa_signal_add_screlease(s, parts); }

void SdmaEngine::wait(hsa_signal_t s) {
  const hsa_signal_value_t v =
      hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  if (v < 0) throw std::runtime_error("SDMA copy reported an error (completion signal < 0)");
}

int SdmaEngine::parts(size_t bytes, int ways) const {
  if (bytes == 0) return 0;
  if (ways < 1) ways = 1;
  const size_t min_part = (size_t)8 << 20;  // smaller parts do not pay for an extra engine
  int n = (int)std::min<size_t>((size_t)ways, (bytes + min_part - 1) / min_part);
  return n < 1 ? 1 : n;
}

int SdmaEngine::copy_d2h(void* dst_host, const void* src_dev, size_t bytes, hsa_signal_t sig, int ways) {
  const int n = parts(bytes, ways);
  if (n == 0) return 0;
  size_t per = (bytes + n - 1) / n;
  per = (per + 4095) & ~(size_t)4095;
  size_t off = 0;
  int issued = 0;
  for (int k = 0; k < n && off < bytes; ++k) {
    const size_t len = std::min(per, bytes - off);
    void* d = static_cast<uint8_t*>(dst_host) + off;
    const void* s = static_cast<const uint8_t*>(src_dev) + off;
    hsa_status_t st = HSA_STATUS_ERROR;
    if (!engine_ids_.empty()) {
      const uint32_t eng = engine_ids_[(size_t)(next_engine_.fetch_add(1) & 0x7fffffff) % engine_ids_.size()];
      st = hsa_amd_memory_async_copy_on_engine(d, cpu_, s, gpu_, len, 0, nullptr, sig,
                                               (hsa_amd_sdma_engine_id_t)eng, false);
    }
    if (st != HSA_STATUS_SUCCESS) st = hsa_amd_memory_async_copy(d, cpu_, s, gpu_, len, 0, nullptr, sig);
    hsa_check(st, "memory_async_copy (D2H)");
    off += len;
    ++issued;
  }
  // parts() may overestimate when the aligned split leaves a part empty: release the surplus
  for (int k = issued; k < n; ++k) hsa_signal_subtract_screlease(sig, 1);
  return n;
}

void SdmaEngine::copy_h2d(void* dst_dev, const void* src_host, size_t bytes, hsa_signal_t sig) {
  hsa_status_t st = HSA_STATUS_ERROR;
  if (h2d_engine_)
    st = hsa_amd_memory_async_copy_on_engine(dst_dev, gpu_, src_host, cpu_, bytes, 0, nullptr, sig,
                                             (hsa_amd_sdma_engine_id_t)h2d_engine_, false);
  if (st != HSA_STATUS_SUCCESS) st = hsa_amd_memory_async_copy(dst_dev, gpu_, src_host, cpu_, bytes, 0, nullptr, sig);
  hsa_check(st, "memory_async_copy (H2D)");
}

std::string SdmaEngine::describe() const {
  std::string e;
  for (auto id : engine_ids_) {
    if (!e.empty()) e += ",";
    int b = 0;
    while (b < 16 && !(id & (1u << b))) ++b;
    e += std::to_string(b);
  }
  int hb = 0;
  while (hb < 16 && !(h2d_engine_ & (1u << hb))) ++hb;
  return "sdma[numa=" + std::to_string(numa_node_) + " engines=" + (e.empty() ? "auto" : e) +
         " h2d=" + (h2d_engine_ ? std::to_string(hb) : std::string("auto")) + "]";
}

}  // namespace gpu
}  // namespace uda
