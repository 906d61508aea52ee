// Node-local registry of GPU work, shared by every libuda process on the machine (the MOFSupplier in
// the NodeManager / TaskTracker, and every reduce task's process).
//
// It answers two questions no single process can answer alone:
//   * placement: which GPU should a new reduce task use? (mapred.uda.gpu.device=auto: the visible
//     GPU with the fewest live reduce tasks, then the fewest HBM bytes in use)
//   * memory: how many HBM bytes do all processes hold on a GPU? (the per-device byte budget,
//     mapred.uda.gpu.hbm.budget, is checked against the node-wide total)
//
// Reference analogue: the reference runs one NetMerger per reduce task process
// (/root/reference/src/Merger/reducer.h:137) and its transport maps every IB device of the node
// (src/DataNet/RDMAComm.cc:156-176), taking the one a connection arrived on (:372-382); its buffers
// are sized from the task's shuffle-memory share (src/Merger/reducer.cc:102-120, 453-496). On an
// MI355X node the scarce shared resources are the GPUs and their HBM, so reduce tasks register
// here and pick the least-loaded GPU; every process publishes the HBM it holds.
//
// One POSIX shared-memory segment (default "/uda_node_v1.<uid>", env UDA_NODE_REGISTRY overrides),
// created by the first process that needs it and never unlinked (it is a few hundred KiB). A robust
// process-shared mutex guards it; entries whose process died (pid gone, or reused: start time
// differs) are reclaimed by the next caller. Devices are named by a key string (the PCI bus id on
// a GPU box), so processes with different HIP_VISIBLE_DEVICES masks agree on which GPU is which.
// Pure host code (no HIP): tested on the CPU tier with real processes.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace uda {

class NodeRegistry {
 public:
  static constexpr int kMaxDevices = 64;
  static constexpr int kMaxSlots = 4096;
  static constexpr int kKeyBytes = 48;
  static constexpr int kTagBytes = 40;

  explicit NodeRegistry(const std::string& name = std::string());
  ~NodeRegistry();
  NodeRegistry(const NodeRegistry&) = delete;
  NodeRegistry& operator=(const NodeRegistry&) = delete;
  // Process-wide registry (default name); nullptr if shared memory is unavailable.
  static NodeRegistry* instance();
  const std::string& name() const { return name_; }

  struct Placement {
    int index = -1;  // into the keys given to place_task
    int slot = -1;   // release(slot) when the task ends
  };
  // Register a reduce task on the device of `keys` with the fewest live tasks (ties: fewest HBM
  // bytes held on the node, then the lowest index).
  Placement place_task(const std::vector<std::string>& keys, const std::string& tag);
  // Register a reduce task on a device chosen by the caller (pinned placement still counts).
  int add_task(const std::string& key, const std::string& tag);
  void release(int slot);

  // HBM bytes this process holds on `key` (one entry per process and device, created on demand);
  // `resident` of them are data that stays (a provider's MOF store), the rest working sets that
  // come and go with tasks.
  void set_bytes(const std::string& key, int64_t bytes, int64_t resident = 0);
  struct Use {
    int tasks = 0;
    int64_t bytes = 0;
    int64_t resident = 0;
  };
  Use usage(const std::string& key);  // every live process on the node
  // Entries of dead processes reclaimed by calls through this handle.
  int64_t reclaimed() const { return reclaimed_; }
  // Remove the segment name (tests); existing mappings stay valid.
  void unlink();

 private:
  struct Header;
  struct Slot;
  struct Lock;
  Header* hdr() const;
  Slot* slots() const;
  int device_index(const std::string& key, bool create);  // under the lock
  void reap();                                             // under the lock
  int take_slot();                                         // under the lock

  std::string name_;
  uint8_t* base_ = nullptr;
  size_t total_ = 0;
  int pid_ = 0;
  uint64_t start_ = 0;
  int64_t reclaimed_ = 0;
  double last_reap_ = 0;
  std::vector<int> my_bytes_slot_;  // per device index: this process's bytes entry (a hint)
};

// Start time of a process (clock ticks since boot, /proc/<pid>/stat field 22); 0 if unknown.
uint64_t process_start_ticks(int pid);
// Live and not a zombie (and, if start != 0, still the same process).
bool process_running(int pid, uint64_t start);

}  // namespace uda
