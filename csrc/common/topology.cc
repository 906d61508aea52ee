// Node topology for host-thread placement. See uda/topology.h.
#include "uda/topology.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <sstream>
#include <tuple>

namespace uda {

namespace {
std::string read_first_line(const std::string& path) {
  std::ifstream f(path);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}
}  // namespace

std::string GpuLocation::bdf() const {
  char b[32];
  std::snprintf(b, sizeof(b), "%04x:%02x:%02x.%x", domain, bus, dev, func);
  return b;
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    while (!tok.empty() && (tok.back() == '\n' || tok.back() == ' ')) tok.pop_back();
    if (tok.empty()) continue;
    int lo = 0, hi = 0;
    if (std::sscanf(tok.c_str(), "%d-%d", &lo, &hi) != 2) hi = lo = std::atoi(tok.c_str());
    for (int c = lo; c <= hi; ++c) v.push_back(c);
  }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  return v;
}

std::string format_cpulist(const std::vector<int>& cpus) {
  std::string out;
  for (size_t i = 0; i < cpus.size();) {
    size_t j = i;
    while (j + 1 < cpus.size() && cpus[j + 1] == cpus[j] + 1) ++j;
    if (!out.empty()) out += ",";
    out += std::to_string(cpus[i]);
    if (j > i) out += "-" + std::to_string(cpus[j]);
    i = j + 1;
  }
  return out;
}

std::string sysfs_root() {
  const char* e = std::getenv("UDA_SYSFS_ROOT");
  return e ? e : "";
}

int pci_numa_node(uint32_t domain, uint32_t bus, uint32_t dev, uint32_t func) {
  char p[96];
  std::snprintf(p, sizeof(p), "/sys/bus/pci/devices/%04x:%02x:%02x.%x/numa_node", domain, bus, dev, func);
  const std::string s = read_first_line(sysfs_root() + p);
  return s.empty() ? -1 : std::atoi(s.c_str());
}

std::vector<GpuLocation> node_gpus() {
  std::vector<GpuLocation> out;
  const std::string dir = sysfs_root() + "/sys/class/kfd/kfd/topology/nodes";
  DIR* d = ::opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::ifstream f(dir + "/" + e->d_name + "/properties");
    if (!f) continue;
    std::string k;
    uint64_t v = 0;
    uint64_t simd = 0, loc = 0, dom = 0;
    int64_t minor = -1;
    bool has_loc = false;
    while (f >> k >> v) {
      if (k == "simd_count") simd = v;
      else if (k == "location_id") loc = v, has_loc = true;
      else if (k == "domain") dom = v;
      else if (k == "drm_render_minor") minor = (int64_t)v;
    }
    if (simd == 0 || !has_loc) continue;  // a CPU node
    GpuLocation g;
    g.domain = (uint32_t)dom;
    g.bus = (uint32_t)(loc >> 8) & 0xFF;
    g.dev = (uint32_t)(loc >> 3) & 0x1F;
    g.func = (uint32_t)loc & 0x7;
    g.numa_node = pci_numa_node(g.domain, g.bus, g.dev, g.func);
    g.render_minor = (int)minor;
    out.push_back(g);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end(), [](const GpuLocation& a, const GpuLocation& b) {
    return std::tie(a.domain, a.bus, a.dev, a.func) < std::tie(b.domain, b.bus, b.dev, b.func);
  });
  return out;
}

std::vector<GpuLocation> usable_gpus() {
  std::vector<GpuLocation> out;
  for (const auto& g : node_gpus()) {
    if (g.render_minor < 0) continue;
    const std::string dev = sysfs_root() + "/dev/dri/renderD" + std::to_string(g.render_minor);
    // open, not access(): a container's device cgroup refuses the other GPUs' nodes only at open
    const int fd = ::open(dev.c_str(), O_RDWR | O_CLOEXEC);
    if (fd >= 0) {
      ::close(fd);
      out.push_back(g);
    }
  }
  return out;
}

std::vector<int> numa_node_cpus(int node) {
  if (node < 0) return {};
  return parse_cpulist(read_first_line(sysfs_root() + "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
}

std::vector<int> allowed_cpus() {
  cpu_set_t s;
  std::vector<int> v;
  if (sched_getaffinity(0, sizeof(s), &s) != 0) return v;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &s)) v.push_back(c);
  return v;
}

std::vector<int> consumer_cpus(const GpuLocation& gpu, const std::vector<GpuLocation>& gpus,
                               const std::vector<int>& allowed) {
  if (gpu.numa_node < 0) return {};
  std::vector<int> cpus = numa_node_cpus(gpu.numa_node);
  if (!allowed.empty()) {
    std::vector<int> x;
    std::set_intersection(cpus.begin(), cpus.end(), allowed.begin(), allowed.end(), std::back_inserter(x));
    cpus.swap(x);
  }
  if (cpus.empty()) return {};
  int k = -1, n = 0;  // this GPU's index among the GPUs of its node
  for (const auto& g : gpus) {
    if (g.numa_node != gpu.numa_node) continue;
    if (g.domain == gpu.domain && g.bus == gpu.bus && g.dev == gpu.dev && g.func == gpu.func) k = n;
    ++n;
  }
  if (k < 0 || n <= 1) return cpus;  // unknown to the topology, or alone on its node: the whole node
  // cut whole cores, not CPU numbers: a core's SMT siblings are numbered far apart (0-63,128-191), and a
  // slice of numbers would hand GPU 0's cores' second threads to GPU 2
  std::vector<std::vector<int>> cores;
  std::vector<char> taken(cpus.empty() ? 0 : (size_t)cpus.back() + 1, 0);
  for (int c : cpus) {
    if (taken[(size_t)c]) continue;
    std::vector<int> sib = parse_cpulist(read_first_line(sysfs_root() + "/sys/devices/system/cpu/cpu" +
                                                         std::to_string(c) + "/topology/thread_siblings_list"));
    std::vector<int> core;
    for (int x : sib)
      if (x < (int)taken.size() && !taken[(size_t)x] && std::binary_search(cpus.begin(), cpus.end(), x)) core.push_back(x);
    if (core.empty() || !std::binary_search(core.begin(), core.end(), c)) core = {c};
    for (int x : core) taken[(size_t)x] = 1;
    cores.push_back(core);
  }
  const size_t per = cores.size() / (size_t)n;
  if (per == 0) return cpus;  // fewer cores than GPUs: sharing beats starving
  const size_t b = (size_t)k * per, e = (k == n - 1) ? cores.size() : b + per;
  std::vector<int> out;
  for (size_t i = b; i < e; ++i) out.insert(out.end(), cores[i].begin(), cores[i].end());
  std::sort(out.begin(), out.end());
  return out;
}

bool bind_thread_to_cpus(const std::vector<int>& cpus) {
  if (cpus.empty()) return true;
  cpu_set_t s;
  CPU_ZERO(&s);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &s);
  return pthread_setaffinity_np(pthread_self(), sizeof(s), &s) == 0;
}

}  // namespace uda
