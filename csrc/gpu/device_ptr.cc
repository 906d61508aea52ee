// Device MOF descriptors: export (provider) and mapping (reducer). See device_ptr.h.
#include "device_ptr.h"

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "device_engine.h"
#include "uda/node_registry.h"

namespace uda {
namespace gpu {

namespace {
std::string to_hex(const void* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) {
    s += d[b[i] >> 4];
    s += d[b[i] & 15];
  }
  return s;
}

bool from_hex(const std::string& s, void* out, size_t n) {
  if (s.size() != 2 * n) return false;
  uint8_t* b = static_cast<uint8_t*>(out);
  for (size_t i = 0; i < n; ++i) {
    unsigned v = 0;
    if (std::sscanf(s.c_str() + 2 * i, "%2x", &v) != 1) return false;
    b[i] = (uint8_t)v;
  }
  return true;
}

std::vector<std::string> split_at(const std::string& s) {
  std::vector<std::string> f;
  size_t b = 0;
  for (;;) {
    const size_t e = s.find('@', b);
    f.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) return f;
    b = e + 1;
  }
}

// Process-wide map of opened IPC handles (a handle is opened once per process). Registered stores
// stay mapped for the process's life; leased ones (a provider HBM store entry) are counted per
// resolved descriptor and closed when the last one is released.
struct Mapping {
  uint8_t* base = nullptr;
  int leased_refs = 0;
  bool leased = false;
};
std::mutex g_ipc_mu;
std::map<std::string, Mapping>& opened() {
  static auto* m = new std::map<std::string, Mapping>();
  return *m;
}
}  // namespace

IpcExport ipc_export(const void* ptr) {
  IpcExport ex;
  ex.handle_hex = "-";
  void* base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)) != hipSuccess || !base) {
    (void)hipGetLastError();
    ex.base = static_cast<const uint8_t*>(ptr);
    return ex;
  }
  ex.base = static_cast<const uint8_t*>(base);
  ex.size = size;
  if (!ipc_size_ok(size)) {  // importing it would hang the reducer: peers fetch bytes instead
    ex.refused = "allocation of " + std::to_string(size) + " bytes is in the hipIpc-hanging size range";
    return ex;
  }
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, base) == hipSuccess)
    ex.handle_hex = to_hex(&h, sizeof(h));
  else
    (void)hipGetLastError();
  return ex;
}

bool ipc_size_ok(size_t bytes) { return ((uint64_t)bytes & 0xFFFFFFFFull) < (1ull << 31); }

const std::string& node_id() {
  // hostname + kernel boot id: two processes may share device memory over hipIpc only when both
  // are equal (same machine, same boot); a container with its own hostname is treated as foreign
  static const std::string id = [] {
    char host[256] = {0};
    (void)gethostname(host, sizeof(host) - 1);
    std::string boot;
    if (FILE* f = std::fopen("/proc/sys/kernel/random/boot_id", "r")) {
      char b[64] = {0};
      if (std::fgets(b, sizeof(b), f)) boot = b;
      std::fclose(f);
    }
    uint64_t h = 1469598103934665603ull;  // FNV-1a
    for (char c : std::string(host) + "|" + boot) h = (h ^ (uint8_t)c) * 1099511628211ull;
    char out[17];
    std::snprintf(out, sizeof(out), "%016llx", (unsigned long long)h);
    return std::string(out);
  }();
  return id;
}

size_t ipc_safe_bytes(size_t bytes) {
  const uint64_t r = (uint64_t)bytes & 0xFFFFFFFFull;
  if (r < (1ull << 31)) return bytes;
  return bytes + ((1ull << 32) - r) + (64ull << 20);  // remainder 64 MiB
}

std::string make_device_descriptor(int device, const uint8_t* ptr, const IpcExport& ipc, bool leased) {
  char head[128];
  std::snprintf(head, sizeof(head), "hbm@%s@%d@%d@%llx@", node_id().c_str(), device, (int)getpid(),
                (unsigned long long)(uintptr_t)ptr);
  return std::string(head) + ipc.handle_hex + "@" + std::to_string((long long)(ptr - ipc.base)) + (leased ? "@L" : "");
}

std::string reducer_holder_id(const std::string& task) {
  const int pid = (int)getpid();
  return node_id() + ":" + std::to_string(pid) + ":" + std::to_string((unsigned long long)process_start_ticks(pid)) +
         ":" + task;
}

int open_ipc_mappings() {
  std::lock_guard<std::mutex> g(g_ipc_mu);
  return (int)opened().size();
}

void release_device_descriptor(const std::string& desc) {
  const auto f = split_at(desc);
  if (f.size() != 8 || f[7] != "L" || f[5] == "-" || std::atoi(f[3].c_str()) == (int)getpid()) return;
  std::lock_guard<std::mutex> g(g_ipc_mu);
  auto it = opened().find(f[5]);
  if (it == opened().end() || !it->second.leased) return;
  if (--it->second.leased_refs > 0) return;
  (void)hipIpcCloseMemHandle(it->second.base);
  (void)hipGetLastError();
  opened().erase(it);
}

bool is_device_descriptor(const std::string& s) { return s.rfind("hbm@", 0) == 0; }

const uint8_t* try_resolve_device_descriptor(const std::string& desc, int my_device, std::string* why) {
  const auto f = split_at(desc);
  if ((f.size() != 7 && !(f.size() == 8 && f[7] == "L")) || f[0] != "hbm") {
    if (why) *why = "malformed device descriptor '" + desc + "'";
    return nullptr;
  }
  if (f[1] != node_id()) {  // another machine (or container): its addresses and handles mean nothing here
    if (why) *why = "descriptor from another node";
    return nullptr;
  }
  const int dev = std::atoi(f[2].c_str());
  const int pid = std::atoi(f[3].c_str());
  const uint8_t* addr = reinterpret_cast<const uint8_t*>((uintptr_t)std::strtoull(f[4].c_str(), nullptr, 16));
  try {
    if (pid == (int)getpid()) {
      if (dev != my_device) {  // same process, other GPU: reads go peer-to-peer over xGMI
        int can = 0;
        HIP_CHECK(hipDeviceCanAccessPeer(&can, my_device, dev));
        if (!can) {
          if (why) *why = "device " + std::to_string(my_device) + " cannot access device " + f[2];
          return nullptr;
        }
        const hipError_t e = hipDeviceEnablePeerAccess(dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
        (void)hipGetLastError();
      }
      return addr;
    }
    if (f[5] == "-") {
      if (why) *why = "provider allocation is not IPC-shareable";
      return nullptr;
    }
    const bool leased = f.size() == 8;
    std::lock_guard<std::mutex> g(g_ipc_mu);
    auto it = opened().find(f[5]);
    if (it == opened().end()) {
      hipIpcMemHandle_t h;
      if (!from_hex(f[5], &h, sizeof(h))) {
        if (why) *why = "bad IPC handle in descriptor";
        return nullptr;
      }
      void* p = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      Mapping mp;
      mp.base = static_cast<uint8_t*>(p);
      mp.leased = leased;
      it = opened().emplace(f[5], mp).first;
    }
    if (leased) it->second.leased_refs++;
    return it->second.base + std::strtoll(f[6].c_str(), nullptr, 10);
  } catch (const std::exception& e) {
    (void)hipGetLastError();  // the caller falls back to bytes: the failed import must not linger
    if (why) *why = e.what();
    return nullptr;
  }
}

const uint8_t* resolve_device_descriptor(const std::string& desc, int my_device) {
  std::string why;
  const uint8_t* p = try_resolve_device_descriptor(desc, my_device, &why);
  if (!p) throw std::runtime_error("cannot map device descriptor: " + why);
  return p;
}

namespace {
std::mutex g_free_mu;
std::atomic<uint64_t> g_free_epoch{0};
std::map<uintptr_t, uint64_t>& freed_bases() {
  static auto* m = new std::map<uintptr_t, uint64_t>();  // base -> epoch of its last free
  return *m;
}
}  // namespace

uint64_t alloc_epoch() { return g_free_epoch.load(std::memory_order_acquire); }

void note_device_free(const void* base) {
  std::lock_guard<std::mutex> g(g_free_mu);
  freed_bases()[(uintptr_t)base] = g_free_epoch.fetch_add(1, std::memory_order_acq_rel) + 1;
}

bool freed_since(const void* base, uint64_t epoch) {
  if (g_free_epoch.load(std::memory_order_acquire) == epoch) return false;  // nothing freed at all
  std::lock_guard<std::mutex> g(g_free_mu);
  auto it = freed_bases().find((uintptr_t)base);
  return it != freed_bases().end() && it->second > epoch;
}

void copy_device_to_host(void* dst, const void* src, int64_t bytes) {
  if (bytes > 0) HIP_CHECK(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
}

}  // namespace gpu
}  // namespace uda
