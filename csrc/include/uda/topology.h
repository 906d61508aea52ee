// Node topology for placing a GPU's host-side threads: which NUMA node each GPU of the node hangs off
// and which CPUs that GPU's consumer threads (the reduce tasks' Java-side stand-ins, the delivery copy
// thread) may run on.
//
// On an 8-GPU MI355X node the GPUs share two (or, in NPS4, eight) NUMA nodes. Every GPU's delivery
// ring lives on its own node (sdma.h), and its consumers read from there; when the four GPUs of a node
// each bound their consumers to the whole node, 4 x 16 reduce tasks (copy + walk threads) contended for
// the same cores and L3 domains. consumer_cpus() gives every GPU a disjoint slice of its node's CPUs
// instead: the node's allowed CPUs in order, cut into as many contiguous pieces as the node has GPUs,
// GPU k of the node (by PCI address) taking piece k -- contiguous CPU numbers share L3 domains on EPYC.
//
// Everything is read from sysfs under UDA_SYSFS_ROOT (default ""), so a test can describe any node:
//   <root>/sys/class/kfd/kfd/topology/nodes/<n>/properties  (GPUs: simd_count > 0, domain, location_id)
//   <root>/sys/bus/pci/devices/<dddd:bb:dd.f>/numa_node
//   <root>/sys/devices/system/node/node<n>/cpulist
// The reference has no counterpart (one CPU reducer per JVM, placed by the OS).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace uda {

struct GpuLocation {
  uint32_t domain = 0, bus = 0, dev = 0, func = 0;
  int numa_node = -1;
  int render_minor = -1;    // /dev/dri/renderD<minor> (KFD drm_render_minor)
  std::string bdf() const;  // "dddd:bb:dd.f"
};

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
std::vector<int> parse_cpulist(const std::string& s);
// {0,1,2,3,8} -> "0-3,8"
std::string format_cpulist(const std::vector<int>& cpus);

std::string sysfs_root();
// Every GPU of the node (KFD topology, independent of HIP_VISIBLE_DEVICES), ordered by PCI address.
std::vector<GpuLocation> node_gpus();
// The GPUs this process can open (a container sees the host's whole KFD topology but only its own
// render nodes), in node_gpus() order -- the devices HIP enumerates, without initialising HIP.
std::vector<GpuLocation> usable_gpus();
// NUMA node of the PCI function (-1 if the host does not say).
int pci_numa_node(uint32_t domain, uint32_t bus, uint32_t dev, uint32_t func);
// CPUs of NUMA node `node` (sysfs cpulist), empty if unknown.
std::vector<int> numa_node_cpus(int node);
// This thread's allowed CPUs (sched_getaffinity).
std::vector<int> allowed_cpus();

// The consumer CPU slice of the GPU at PCI address `gpu` among `gpus` (usable_gpus()): the allowed CPUs of
// its NUMA node cut into one contiguous piece per GPU of that node. Empty if the node is unknown (the
// caller then leaves the threads unbound). `allowed` empty = no restriction.
std::vector<int> consumer_cpus(const GpuLocation& gpu, const std::vector<GpuLocation>& gpus,
                               const std::vector<int>& allowed);

// Bind the calling thread to `cpus` (no-op when empty); false if the kernel refused.
bool bind_thread_to_cpus(const std::vector<int>& cpus);

}  // namespace uda
