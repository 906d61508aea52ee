// Provider HBM store for Hadoop-written map output files (the MOFs found through getPathUda).
//
// Reference: the DataEngine resolves (job, map, reduce) through getPathUda on first touch and then
// reads the partition chunk by chunk from the MOF file with O_DIRECT AIO for every request
// (src/MOFServer/IndexInfo.cc:238-274 process_shuffle_request, :304-335 aio_read_chunk_data); its
// fd cache is refcounted by in-flight reads (:195-233) and a chunk is released only when the SEND
// that used it completed (:276-301, src/DataNet/RDMAServer.cc:200-213).
//
// MI355X design: the first descriptor fetch that touches a MOF file makes it resident in HBM (an
// allocation of its own, exportable over hipIpc); every fetch of any of its partitions is answered
// with a device descriptor, so reducers on the node merge the partitions where they lie (xGMI
// reads from another GPU) and the file is read from disk once instead of once per reducer.
//
// Loading: one loader thread per GPU, each with its own io_uring reads (O_DIRECT, 4 KiB aligned)
// into a pinned chunk ring on that GPU's NUMA node and SDMA H2D copies. A loader reads the chunks of
// every file it is loading in turn, so all files of a job advance together; since a MOF holds its
// partitions in order, partition r of every file lands at about the same time and reduce task r
// can start as soon as its partitions are in (a fetch is answered once the bytes up to the end of
// its partition have landed, not the whole file).
//
// Lifetime: a descriptor handed out is a reference, held by the reducer that fetched it (holder id:
// node, pid, process start time, task) until it releases it -- when its merge has consumed the
// partitions, or when the task ends or fails. An entry with holders is never evicted, whatever the
// budget pressure; entries of finished jobs (JOB_OVER) go first, then unreferenced ones by LRU.
// Backstop for reducers that die without releasing: a holder on this node whose process is gone is
// dropped; a holder on another node that has not fetched from the entry for `lease_s` is dropped.
// When the budget is exhausted and nothing is evictable, the fetch is declined ("not device
// resident") and the reducer fetches the partition's bytes instead: never a wrong answer.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "device_ptr.h"

namespace uda {
class AsyncIO;
namespace gpu {

class DeviceBuffer;

class MofCache {
 public:
  struct Options {
    int64_t capacity = 0;           // HBM bytes over all devices (mapred.uda.provider.hbm.bytes); 0 = off
    std::vector<int> devices{0};    // GPUs the MOFs are striped over (mapred.uda.provider.hbm.devices)
    int64_t chunk_bytes = 16 << 20;  // disk read granule
    int chunks = 16;                 // reads + copies in flight per loader
    int64_t read_bytes = 0;          // disk request size a chunk is read in (0: one read per chunk)
    bool odirect = true;
    // a file whose pages are already in the page cache (map outputs written moments ago) is read through
    // it instead of with O_DIRECT (mapred.uda.provider.hbm.cached.read)
    bool cached_read = true;
    double lease_s = 600;            // a holder on another node idle this long is presumed dead
    // An unreferenced entry is evicted to admit another file of ITS OWN job only after this many seconds
    // without a fetch (mapred.uda.provider.hbm.idle.evict.s; 0: plain LRU). A job whose MOFs outgrow the
    // store reads them in waves of reduce tasks, each wave every file in order: LRU then evicted the files
    // the next wave starts with to load the ones it ends with, and reloaded 15 GB of a 20 GB store every
    // wave (r6 node run, 62 GB of MOFs). Entries of finished jobs, of other jobs and of dead holders go
    // as before.
    double idle_evict_s = 0;
  };
  struct Ref {
    const uint8_t* data = nullptr;  // device address of the file's first byte
    int64_t len = 0;                // file size
    int device = -1;
    IpcExport ipc;
  };
  struct Stats {
    int64_t loads = 0, hits = 0, declined = 0, evictions = 0, bytes_loaded = 0, resident_bytes = 0;
    int64_t cached_reads = 0;  // files read through the page cache (Options::cached_read)
    int64_t holders = 0, holders_reaped = 0, releases = 0;
    double load_ms = 0;       // summed per-file load time
    double load_wall_ms = 0;  // time any load was in progress (loads overlap)
    double open_ms = 0;       // summed HBM allocation + IPC export + open of new entries
    double open_alloc_ms = 0, open_export_ms = 0;  // the allocation and export parts of open_ms
    double open_file_ms = 0, open_file_max_ms = 0;  // open(2) of the files: summed, slowest
    // CLOCK_BOOTTIME ms (the task processes' clock) of the first miss, the first disk read issued and
    // the latest file fully landed: the loads' place on a wave's timeline
    double first_miss_boot_ms = 0, first_read_boot_ms = 0, last_landed_boot_ms = 0;
  };
  // ok: the bytes [0, need_end) are in HBM (ref valid); else why says what failed.
  using Ready = std::function<void(bool ok, const Ref& ref, const std::string& why)>;

  explicit MofCache(const Options& o);
  ~MofCache();
  MofCache(const MofCache&) = delete;
  MofCache& operator=(const MofCache&) = delete;

  bool enabled() const { return opt_.capacity > 0 && !opt_.devices.empty(); }
  // Start every device's loader now (its I/O ring, pinned staging, SDMA signals) instead of at the
  // first file: a node daemon does this at start, off the first wave's critical path.
  void start_loaders();
  int64_t capacity() const { return opt_.capacity; }
  // Take `holder`'s reference on the MOF file `path` of job `job` (loading it on first touch) and
  // call ready() once its first need_end bytes are resident: inline if they already are, else from
  // a loader thread. false (reason in *why; ready never called) when it cannot be cached now.
  bool acquire_async(const std::string& job, const std::string& path, const std::string& holder, int64_t need_end,
                     Ready ready, std::string* why);
  // Blocking form (tests): the whole file.
  bool acquire(const std::string& job, const std::string& path, const std::string& holder, Ref* out, std::string* why);
  // Drop one of holder's references on `path` / all of holder's references on job's MOFs (job "*": on
  // every job's).
  void release(const std::string& path, const std::string& holder);
  void release_holder(const std::string& job, const std::string& holder);
  // The job is over: its MOFs may be evicted at once, whoever still holds them.
  void job_over(const std::string& job);
  // The hipIpc export of a loaded file's HBM, made on first need and kept with the entry: a reducer in
  // this process (a task hosted by the node daemon) reads the memory directly, so the export (a dmabuf,
  // ~4.4 ms per 1.3 GB file, serialized in the runtime) is paid only when another process maps it.
  // An entry gone meanwhile: an export without a handle (the reducer fetches bytes).
  IpcExport export_of(const std::string& path);
  Stats stats();

 private:
  struct Waiter {
    int64_t need_end;
    Ready ready;
  };
  struct Entry {
    std::string job, path;
    int device = -1;
    int64_t len = 0;
    std::unique_ptr<DeviceBuffer> mem;
    const uint8_t* dptr = nullptr;
    IpcExport ipc;        // handle "-" until export_of() made it
    bool exported = false;
    std::mutex export_mu;  // one export per entry
    bool loading = true, failed = false, job_done = false;
    std::string error;
    double last_served = 0, t_start = 0;
    std::map<std::string, std::pair<int, double>> holders;  // holder -> (references, last fetch time)
    std::vector<Waiter> waiters;
    // loader state
    int fd = -1;
    bool direct = false;
    int64_t next_read = 0, landed = 0;
    std::map<int64_t, int64_t> done_chunks;  // landed beyond `landed`: offset -> length
    int reads_in_flight = 0;
  };
  bool eager_export_ = false;  // UDA_STORE_EAGER_EXPORT=1: export every entry when it is allocated
  struct Loader;
  struct Fire {
    Ready ready;
    bool ok;
    Ref ref;
    std::string why;
  };

  // mu_ held: evict until `bytes` fit (for a file of `job`)
  bool make_room(int device, int64_t bytes, double now, const std::string& job);
  bool evictable(Entry& e, double now);                   // mu_ held (reaps dead holders)
  void erase_entry(const std::string& path);              // mu_ held
  Ref ref_of(const Entry& e) const;
  void loader_main(Loader* L);
  void opener_main(Loader* L);
  Loader* loader_locked(int device);  // the device's loader, started on first use (mu_ held)
  void fail_entry(Entry& e, const std::string& why, std::vector<Fire>* fire);  // mu_ held
  void collect_ready(Entry& e, std::vector<Fire>* fire);                      // mu_ held

  Options opt_;
  int64_t per_device_ = 0;
  std::mutex mu_;
  std::map<std::string, std::shared_ptr<Entry>> entries_;  // by path
  std::map<int, int64_t> used_;                             // device -> bytes resident or loading
  std::map<int, std::unique_ptr<Loader>> loaders_;          // by device
  Stats st_;
  int busy_loaders_ = 0;
  double busy_since_ = 0;
};

}  // namespace gpu
}  // namespace uda
