// Explicit SDMA (copy-engine) transfers and NUMA-local pinned host memory for the delivery path.
//
// Why not hipMemcpyAsync: for device -> pinned-host copies the HIP runtime passes the GPU agent as
// both source and destination agent, and ROCr then runs the copy as a blit *kernel*
// (__amd_rocclr_copyBuffer) on the CUs — it competes with the merge kernels for the very CUs the
// merge needs (round-1 profile: 52% of GPU time in 512 MiB blits). Here the copy is issued with
// the CPU agent as destination agent on an explicitly chosen SDMA engine, so delivery runs on the
// copy engines and the CUs stay with the merge.
//
// The pinned ring is carved from the system memory pool of the CPU agent nearest to the GPU
// (HSA_AMD_AGENT_INFO_NEAREST_CPU), i.e. the GPU's local NUMA node, and made accessible to the GPU.
//
// Reference role: the registered RDMA buffers the merged KV stream is staged in before dataFromUda
// (src/Merger/reducer.cc:303-324 kv pool, src/Merger/MergeManager.cc:155-182).
#pragma once
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace uda {
namespace gpu {

class SdmaEngine {
 public:
  // Process-wide engine of a device (created on first use, never destroyed): reduce tasks of one
  // process share the device's delivery engine and its cache of pinned ring blocks.
  static SdmaEngine& for_device(int device);
  // `device` is a HIP ordinal; the HSA GPU agent is matched by PCI domain/BDF.
  explicit SdmaEngine(int device);
  ~SdmaEngine();
  SdmaEngine(const SdmaEngine&) = delete;
  SdmaEngine& operator=(const SdmaEngine&) = delete;

  // Pinned host memory on the GPU's nearest NUMA node, accessible to the GPU (SDMA target).
  void* alloc_host(size_t bytes);
  void free_host(void* p);
  // Cached variant for per-task rings: blocks of exactly `bytes` are reused after release_ring().
  void* acquire_ring(size_t bytes);
  void release_ring(void* p, size_t bytes);

  // Completion signal (value counts outstanding copies; 0 = done).
  hsa_signal_t make_signal();
  void destroy_signal(hsa_signal_t s);
  // Device -> host copy of `bytes`, split over up to `ways` engines; `sig` must hold the number of
  // parts this call adds (use arm()): returns the number of parts issued.
  int copy_d2h(void* dst_host, const void* src_dev, size_t bytes, hsa_signal_t sig, int ways);
  // Parts copy_d2h(bytes, ways) will issue.
  int parts(size_t bytes, int ways) const;
  // Host -> device copy (one part) on an SDMA engine other than the delivery engine when the device
  // has one, so staging from pinned DRAM and D2H delivery use the two directions of the link at once.
  void copy_h2d(void* dst_dev, const void* src_host, size_t bytes, hsa_signal_t sig);
  static void arm(hsa_signal_t s, int64_t parts);
  // Count `parts` more outstanding copies on a signal that may already have some in flight.
  static void add(hsa_signal_t s, int64_t parts);
  // Block until the signal reaches 0; throws on a copy error (negative value).
  static void wait(hsa_signal_t s);

  // One small copy in each direction on the engines this class uses: the runtime creates an engine's
  // queue at its first copy (a cold reduce task's first staging copies waited ~150 ms behind it), so a
  // prewarm can take that cost before the task's data arrives. Synchronous; `dev_scratch` >= 4 KiB.
  void warm(void* dev_scratch);
  int numa_node() const { return numa_node_; }
  int engines() const { return (int)engine_ids_.size(); }
  std::string describe() const;

 private:
  hsa_agent_t gpu_{}, cpu_{};
  hsa_amd_memory_pool_t host_pool_{};
  std::vector<uint32_t> engine_ids_;  // SDMA engine bits usable for CPU <- GPU copies
  uint32_t h2d_engine_ = 0;           // SDMA engine bit for GPU <- CPU staging (0: runtime's choice)
  int numa_node_ = -1;
  std::atomic<int> next_engine_{0};
  bool hsa_inited_ = false;
  std::mutex ring_mu_;
  std::multimap<size_t, void*> ring_cache_;
};

// Linux NUMA node of the HIP device (sysfs), -1 if unknown; and pinning the calling thread to the
// CPUs of that node (no-op when unknown). Used for the delivery/consumer threads.
int device_numa_node(int device);
void bind_thread_to_numa(int node);
// The CPUs the host-side consumer threads of `device` run on: its disjoint slice of its NUMA node's CPUs
// among the node's GPUs (uda/topology.h consumer_cpus); UDA_CONSUMER_CPUS=node: the whole NUMA node
// (every GPU of the node shares it); empty if the topology is unknown.
std::vector<int> device_consumer_cpus(int device);
// Pinned host memory, preferably on NUMA node `node` (< 0: anywhere). Pages are created by the
// caller's threads, not under the runtime's registration: mmap, MADV_HUGEPAGE, first touch from up to
// 8 threads, then hipHostRegister (8 x 256 MiB: ~30 ms, against ~400 ms of hipHostMalloc, which zeroes
// and pins 4 KiB pages one allocation at a time; tools/probes/pinned_alloc_probe.cc). Falls back to
// hipHostMalloc (UDA_PINNED_REGISTER=0, or if the registered range is not mapped at the same device
// address). Free with pinned_host_free.
void* pinned_host_alloc(size_t bytes, int node = -1);
void pinned_host_free(void* p);
// The same, kept for its callers (placement on `node`).
void* hip_host_alloc_on_node(size_t bytes, int node);
// Node merge service (csrc/service/merge_service.h): pinned host memory allocated after
// set_pinned_shareable(true) lives in memfd-backed shared mappings, so a client process can map the
// delivery rings the service's SDMA engine writes and read the merged buffers in place.
// pinned_share_of finds the shareable region holding [p, p + len): its memfd (owned by the region,
// valid while the region is allocated), a process-unique id, the region's size and p's offset in it.
struct PinnedShare {
  int fd = -1;
  uint64_t id = 0;
  size_t offset = 0, region_bytes = 0;
  int numa_node = -1;  // where the pages live (-1: unknown)
};
void set_pinned_shareable(bool on);
bool pinned_share_of(const void* p, size_t len, PinnedShare* out);
// Where the pages of the mapping containing `p` live, from /proc/self/numa_maps: "N1=100%" style
// summary (or "unknown").
std::string numa_residency(const void* p);

}  // namespace gpu
}  // namespace uda
