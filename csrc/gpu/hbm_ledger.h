// Per-device HBM byte budget (mapred.uda.gpu.hbm.budget), shared by everything libuda allocates on a
// GPU -- pooled merge workspaces, the reduce tasks running now, the provider's MOF store -- and by
// every libuda process on the node (the node registry carries each process's bytes).
//
// Reference analogue: the reference sizes every reduce task's buffers from its share of the shuffle
// memory and fails cleanly when they cannot fit (src/Merger/reducer.cc:102-120 handle_init_msg,
// :453-496 calculateMemPool). Here the shared resource is a GPU's 288 GB of HBM3E and the tasks
// sharing it come and go, so a task asks for its working set before its merge starts:
//   * reserve(): waits (FIFO within the process) until the bytes fit under the budget, after first
//     trimming idle pooled objects, largest first; the thread's allocations then draw from it;
//   * headroom(): the largest working set that could ever be granted, so a task that cannot fit
//     shrinks its key-range round (or takes the hybrid path) instead of growing past the budget.
// Every DeviceBuffer allocation and free goes through on_alloc / on_free, so used() is exact for
// this process. An allocation outside a reservation that would exceed the budget trims the pools
// first and is counted (and logged) if it still does not fit: the budget bounds admission, it does
// not turn a running task's allocation into a failure.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <string>
#include <vector>
#include <deque>

namespace uda {
namespace gpu {

// Node-registry key of a HIP device (its PCI bus id; stable across HIP_VISIBLE_DEVICES masks) and
// the keys of every device this process sees.
std::string device_key(int device);
std::vector<std::string> visible_device_keys();

class HbmLedger {
 public:
  static HbmLedger& get();

  // conf value: bytes (> 1) or a fraction of the device's HBM (0 < f <= 1); <= 0: kDefaultFraction.
  static constexpr double kDefaultFraction = 0.92;
  void configure(int device, double conf);
  int64_t budget(int device);

  // resident: data that stays (a MOF store), not a task's working set
  void on_alloc(int device, int64_t bytes, bool resident = false);
  void on_free(int device, int64_t bytes, bool resident = false);

  class Reservation {
   public:
    ~Reservation();
    Reservation(const Reservation&) = delete;
    Reservation& operator=(const Reservation&) = delete;
    int device() const { return device_; }
    int64_t granted() const { return granted_; }
    int64_t left() const { return left_; }
    double wait_ms() const { return wait_ms_; }
    // make the reservation the one this thread's allocations draw from (the creating thread binds
    // automatically); the returned scope unbinds
    struct Scope {
      explicit Scope(Reservation* p) : prev(p) {}
      Scope(const Scope&) = delete;
      Scope& operator=(const Scope&) = delete;
      ~Scope();
      Reservation* prev;
    };
    Scope bind();
    // stop being the creating thread's reservation (it is handed to other threads with bind())
    void unbind();

   private:
    friend class HbmLedger;
    Reservation() = default;
    int device_ = 0;
    int64_t granted_ = 0;
    int64_t left_ = 0;
    double wait_ms_ = 0;
    Reservation* prev_bound_ = nullptr;
  };
  // Wait until `bytes` more fit under the device's budget (node-wide), trimming idle pools first.
  // Throws HbmBudgetError (uda/error.h) when `bytes` exceed headroom(), on timeout, or when stop()
  // turns true. bytes <= 0: an empty reservation, granted at once.
  std::unique_ptr<Reservation> reserve(int device, int64_t bytes, const std::function<bool()>& stop = nullptr,
                                       double timeout_s = 1800);
  // The reservation this thread's allocations draw from (nullptr: none).
  Reservation* bound();
  int64_t used(int device);  // this process
  // Largest reservation that could be granted once every other task of this process has finished
  // and every idle pooled object is freed: budget - (bytes other processes hold) - (bytes this
  // process holds that are neither idle in a pool nor reserved by a running task).
  int64_t headroom(int device);

  // Idle pooled device objects: trim(device, want) frees up to `want` bytes (largest first) and
  // returns what it freed; idle(device) reports the bytes it could free.
  struct Pool {
    std::function<int64_t(int, int64_t)> trim;
    std::function<int64_t(int)> idle;
  };
  void add_pool(Pool p);

  struct Stats {
    int64_t budget = 0, used = 0, reserved = 0, peak = 0, resident = 0, node_bytes = 0, trimmed = 0, over = 0;
    int64_t device_peak = 0;  // device-reported HBM in use, highest seen at a reservation
    int64_t waits = 0;
    double wait_ms = 0;
  };
  Stats stats(int device);
  // Start a new peak window (benchmarks: the peak of one timed step, not of the setup before it).
  void reset_peak(int device);
  // Tests: account allocations of a device without touching HIP (fake HBM size and key).
  void set_fake_device(int device, int64_t total_bytes, const std::string& key);
  // Tests: device memory a fake device reports in use beyond what the ledgers track (HIP runtime, code
  // objects, allocations outside libuda).
  void set_fake_untracked(int device, int64_t bytes);

 private:
  HbmLedger() = default;
  struct Dev {
    bool init = false;
    std::string key;  // node-registry key (PCI bus id)
    int64_t total = 0, budget = 0;
    bool fake = false;  // set_fake_device: no HIP device behind it
    int64_t fake_untracked = 0;  // set_fake_untracked
    int64_t used = 0, reserved = 0, peak = 0, resident = 0, trimmed = 0, over = 0, waits = 0;
    int64_t device_peak = 0;  // HBM in use on the device (hipMemGetInfo) seen at reservations
    double wait_ms = 0;
    uint64_t next_ticket = 0;
    std::deque<uint64_t> queue;  // reservations waiting, FIFO
  };
  Dev& dev(int device);  // mu_ held
  void publish(Dev& d);  // mu_ held: this process's bytes into the node registry
  int64_t others(Dev& d);  // mu_ held: bytes the node's other processes hold
  int64_t others_resident(Dev& d);  // mu_ held: resident bytes of the node's other processes
  int64_t device_used(int device, Dev& d);  // HBM in use on the device, tracked or not (0 if unknown)
  int64_t untracked(int device, Dev& d);    // mu_ held: device HBM in use that no process's ledger counts
  int64_t trim_pools(int device, int64_t want);  // mu_ NOT held
  int64_t idle_bytes(int device);                // mu_ NOT held

  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int, Dev> devs_;
  std::mutex pools_mu_;
  std::vector<Pool> pools_;
};

}  // namespace gpu
}  // namespace uda
