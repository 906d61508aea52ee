// Provider HBM store for Hadoop-written map output files (the MOFs found through getPathUda).
//
// Reference: the DataEngine resolves (job, map, reduce) through getPathUda on first touch and then
// reads the partition chunk by chunk from the MOF file with O_DIRECT AIO for every request
// (src/MOFServer/IndexInfo.cc:238-274 process_shuffle_request, :304-335 aio_read_chunk_data).
//
// MI355X design: on the first descriptor fetch that touches a MOF file, the whole file is read once
// (io_uring O_DIRECT into a NUMA-local pinned chunk ring, a window of reads in flight) and copied
// into an HBM allocation of its own (hipMemcpyAsync per chunk, i.e. the SDMA engines), exportable
// over hipIpc. Every later fetch of any of its partitions is answered with a device descriptor, so
// reducers on the node merge the partitions where they lie (xGMI reads from another GPU) and the
// file is read from disk once instead of once per reducer. MOFs are striped over the configured
// GPUs (the one with the most free budget takes the next file).
//
// Lifetime: a reducer may read a served partition long after the descriptor went out (there is no
// release message in the protocol), so an entry is evictable only when its job ended (JOB_OVER from
// the provider plugin) or when it has not been served for `lease_s` seconds. When the budget is
// exhausted and nothing is evictable, acquire() declines and the provider answers "not device
// resident": the reducer falls back to byte fetches from the file (never a wrong answer).
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "device_ptr.h"

namespace uda {
class AsyncIO;
namespace gpu {

class MofCache {
 public:
  struct Options {
    int64_t capacity = 0;           // HBM bytes over all devices (mapred.uda.provider.hbm.bytes); 0 = off
    std::vector<int> devices{0};    // GPUs the MOFs are striped over (mapred.uda.provider.hbm.devices)
    int64_t chunk_bytes = 16 << 20;  // disk read granule
    int chunks = 8;                  // reads in flight
    bool odirect = true;
    double lease_s = 600;            // an entry served within this many seconds is never evicted
  };
  struct Ref {
    const uint8_t* data = nullptr;  // device address of the file's first byte
    int64_t len = 0;                // file size
    int device = -1;
    IpcExport ipc;
  };
  struct Stats {
    int64_t loads = 0, hits = 0, declined = 0, evictions = 0, bytes_loaded = 0, resident_bytes = 0;
    double load_ms = 0;
  };

  explicit MofCache(const Options& o);
  ~MofCache();
  MofCache(const MofCache&) = delete;
  MofCache& operator=(const MofCache&) = delete;

  bool enabled() const { return opt_.capacity > 0 && !opt_.devices.empty(); }
  // Device copy of the MOF file `path` of job `job` (loaded on first touch; concurrent callers of a
  // file being loaded wait for it). false (reason in *why) when it cannot be cached now.
  bool acquire(const std::string& job, const std::string& path, Ref* out, std::string* why);
  // The job is over: its MOFs may be evicted at once.
  void job_over(const std::string& job);
  Stats stats();

 private:
  struct Entry {
    std::string job;
    int device = -1;
    int64_t len = 0;
    void* dptr = nullptr;
    IpcExport ipc;
    bool loading = true, failed = false, job_done = false;
    std::string error;
    double last_served = 0;
  };
  void load(const std::string& path, Entry* e);  // fills e (device chosen by the caller), throws
  bool make_room(int device, int64_t bytes, double now);  // under mu_: evict until `bytes` fit
  void free_entry(Entry* e);

  Options opt_;
  int64_t per_device_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::shared_ptr<Entry>> entries_;  // by path
  std::map<int, int64_t> used_;                             // device -> bytes resident or loading
  Stats st_;
  // loader state (one load at a time: the disk / PCIe link is the bound, not the CPU)
  std::mutex load_mu_;
  std::unique_ptr<AsyncIO> aio_;
  uint8_t* ring_ = nullptr;
  std::vector<hipEvent_t> ev_;
  std::vector<hipStream_t> streams_;  // per device index
};

}  // namespace gpu
}  // namespace uda
