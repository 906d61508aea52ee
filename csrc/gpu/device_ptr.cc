// Device MOF descriptors: export (provider) and mapping (reducer). See device_ptr.h.
#include "device_ptr.h"

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <vector>

#include "device_engine.h"

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

// Process-wide map of opened IPC handles (a handle is opened once per process).
std::mutex g_ipc_mu;
std::map<std::string, uint8_t*>& opened() {
  static auto* m = new std::map<std::string, uint8_t*>();  // mappings live until process exit
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
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, base) == hipSuccess)
    ex.handle_hex = to_hex(&h, sizeof(h));
  else
    (void)hipGetLastError();
  return ex;
}

size_t ipc_safe_bytes(size_t bytes) {
  const uint64_t r = (uint64_t)bytes & 0xFFFFFFFFull;
  if (r < (1ull << 31)) return bytes;
  return bytes + ((1ull << 32) - r) + (64ull << 20);  // remainder 64 MiB
}

std::string make_device_descriptor(int device, const uint8_t* ptr, const IpcExport& ipc) {
  char head[96];
  std::snprintf(head, sizeof(head), "hbm@%d@%d@%llx@", device, (int)getpid(),
                (unsigned long long)(uintptr_t)ptr);
  return std::string(head) + ipc.handle_hex + "@" + std::to_string((long long)(ptr - ipc.base));
}

bool is_device_descriptor(const std::string& s) { return s.rfind("hbm@", 0) == 0; }

const uint8_t* resolve_device_descriptor(const std::string& desc, int my_device) {
  const auto f = split_at(desc);
  if (f.size() != 6 || f[0] != "hbm") throw std::runtime_error("bad device descriptor '" + desc + "'");
  const int dev = std::atoi(f[1].c_str());
  const int pid = std::atoi(f[2].c_str());
  const uint8_t* addr = reinterpret_cast<const uint8_t*>((uintptr_t)std::strtoull(f[3].c_str(), nullptr, 16));
  if (pid == (int)getpid()) {
    if (dev != my_device) {  // same process, other GPU: reads go peer-to-peer over xGMI
      int can = 0;
      HIP_CHECK(hipDeviceCanAccessPeer(&can, my_device, dev));
      if (!can) throw std::runtime_error("device " + std::to_string(my_device) + " cannot access device " + f[1]);
      const hipError_t e = hipDeviceEnablePeerAccess(dev, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
      (void)hipGetLastError();
    }
    return addr;
  }
  if (f[4] == "-") throw std::runtime_error("provider allocation is not IPC-shareable: " + desc);
  std::lock_guard<std::mutex> g(g_ipc_mu);
  auto it = opened().find(f[4]);
  if (it == opened().end()) {
    hipIpcMemHandle_t h;
    if (!from_hex(f[4], &h, sizeof(h))) throw std::runtime_error("bad IPC handle in descriptor");
    void* p = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    it = opened().emplace(f[4], static_cast<uint8_t*>(p)).first;
  }
  return it->second + std::strtoll(f[5].c_str(), nullptr, 10);
}

void copy_device_to_host(void* dst, const void* src, int64_t bytes) {
  if (bytes > 0) HIP_CHECK(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
}

}  // namespace gpu
}  // namespace uda
