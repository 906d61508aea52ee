// NetMerger reduce task: INIT/FETCH/FINAL/EXIT handling, memory planning, fetch phase, online and
// hybrid (LPQ/RPQ with local-dir spill) merge, delivery to the host through dataFromUda.
//
// Parity:
//   handle_init_msg / reduce_downcall_handler / calculateMemPool (src/Merger/reducer.cc:56-217, 453-496)
//   merge_do_fetching_phase / merge_do_merging_phase / merge_online / fetch_lpqs / merge_hybrid
//   (src/Merger/MergeManager.cc:47-314)
// Backends: "cpu" (heap k-way merge, the reference algorithm) and "gpu" (whole partitions staged in
// HBM and merged by the HIP merge tree; csrc/consumer/gpu_merge.cc), chosen with
// mapred.uda.merge.backend.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "uda/cmd.h"
#include "uda/codec.h"
#include "uda/compare.h"
#include "uda/host.h"
#include "uda/ifile.h"
#include "uda/transport.h"

namespace uda {

class MofFetcher;
namespace gpu {
class DeviceBuffer;
}

// Map task id of a map attempt id (drops the trailing "_<attempt>").
std::string map_task_of(const std::string& attempt);

// A node daemon hosting reduce tasks' merges (service/node_daemon.h) builds once, at its start, what
// each hosted task's GPU prewarm would build on the first wave's critical path: the device's code
// objects and SDMA queues, and `tasks` pooled merge workspaces with their pinned delivery rings (rounds
// of `round_bytes`, `maps` runs, dataFromUda buffers of `kv_buf` bytes). Throws on failure.
void prewarm_node_merges(int device, int tasks, int64_t round_bytes, int maps, int64_t kv_buf);

struct ReduceStats {
  int64_t maps_fetched = 0;
  int64_t bytes_fetched = 0;      // partition bytes received (compressed if compressed)
  int64_t bytes_delivered = 0;    // merged bytes handed to the host
  int64_t records = 0;
  int64_t buffers = 0;
  int64_t lpqs = 0;
  int64_t spill_bytes = 0;
  double fetch_ms = 0, merge_ms = 0, total_ms = 0;
  double wait_ms = 0;             // time the merge waited on the network (total_wait_mem_time)
  int64_t device_decoded_blocks = 0;  // compressed blocks decoded in HBM by the F6 kernels
  int64_t rpq_rounds = 0;             // GPU hybrid: key-range rounds of the RPQ merge; device fetch: merge rounds
  int64_t hybrid_direct = 0;          // GPU hybrid: RPQ rounds straight over the fetched partitions (no LPQ level)
  int64_t merge_budget_from_ledger = 0;  // staged path: input budget capped by the HBM ledger's headroom
  int64_t gpu_ws_bytes = 0;           // device fetch, generic keys: HBM held by the merge workspaces
  // GPU backend phase split: H2D staging, device decode+merge, waits on D2H pieces, host consumers
  // (dataFromUda / spill writes) of the pinned pieces
  double gpu_h2d_ms = 0, gpu_device_ms = 0, gpu_d2h_wait_ms = 0, gpu_sink_ms = 0;
  double gpu_decode_ms = 0;  // device fetch, compressed partitions: framing walk + F6 decode (stream synced)
  double gpu_gate_wait_ms = 0;  // waiting for a GPU merge slot (mapred.uda.gpu.max.concurrent.merges)
  double hbm_wait_ms = 0;       // waiting for the device working set under the HBM budget
  int64_t hbm_reserved = 0;     // bytes of that reservation
  int64_t round_bytes = 0;      // device fetch: key-range round size used (halved to fit the budget)
  int gpu_device = -1;          // HIP device the task ran on (mapred.uda.gpu.device, auto = placed)
  double gpu_prewarm_ms = -1;   // INIT-time GPU prewarm (mapred.uda.gpu.prewarm); -1: not run
  double gpu_prewarm_wait_ms = 0;  // the merge waiting for the prewarm to finish
  std::string gpu_prewarm_phases;  // ms per prewarm phase: hip init, sdma, code, workspaces, fixed10, pinned
  // per-MOF buffer pair split when compressed (reducer.cc:463-491): fetch side / uncompressed side
  int64_t fetch_buf_bytes = 0, uncomp_buf_bytes = 0;
  int64_t restored_lpqs = 0, restored_maps = 0;  // hybrid resume from an LPQ checkpoint
  int64_t device_descriptors = 0;     // GPU device fetch: partitions merged in the provider's HBM
  int64_t unmapped_descriptors = 0;   // descriptors not mappable here (other node, no handle): bytes fetched
  std::string unmapped_reason;        // why the first of them could not be mapped
  double descriptor_map_ms = 0;       // resolving descriptors (hipIpcOpenMemHandle of another process's HBM)
  double fetch_cmd_wait_ms = 0;       // device fetch: waiting for the host's FETCH commands
  double fetch_ack_wait_ms = 0;       // device fetch: waiting for the providers' descriptor answers
  double merge_start_boot_ms = 0;     // device fetch: CLOCK_BOOTTIME ms when the merge began / sent its
  double fetch_sent_boot_ms = 0;      // first descriptor requests (a wave's timeline, bench.py --node)
  double first_data_ms = -1;          // device fetch: from the merge's start to the first dataFromUda
  int64_t host_fetched_bytes = 0;     // GPU device fetch: bytes of MOFs that were not device-resident
  int64_t local_read_bytes = 0;       // of those: read from the MOF files on this node (not over the network)
  std::string merge_path;             // which merge ran ("device-fixed10", "device-generic", ...)
  std::string backend;
};

// A declined partition read in place of fetching it (device fetch, mapred.uda.gpu.fetch.local.read): the
// provider host spec ("host[:port]") names this node, and the MOF file the provider named is a regular file
// (not a symlink) of this process's user holding [off, off + len) -- the descriptor open for reading, or -1.
bool mof_host_is_local(const std::string& host_spec);
int open_local_mof(const std::string& path, int64_t off, int64_t len);

// File confinement of a reduce task that runs on behalf of another local user (a merge-service session
// whose client's uid is not the service's): what the task creates, reads back and unlinks must stay in the
// node's own local directories, and it trusts only files this process's user owns.
struct TaskSandbox {
  bool enabled = false;
  std::vector<std::string> roots;  // canonical local directories a confined task may use (its local_dirs)
};
// Returns "" if `p` (canonicalised) lies inside one of `roots`, else why not.
std::string sandbox_check_dir(const std::vector<std::string>& roots, const std::string& p);
// A file the task may read back / unlink: a regular file (not a symlink) owned by this process's euid
// inside one of `dirs`.
bool sandbox_trusted_file(const std::vector<std::string>& dirs, const std::string& path);

class ReduceTask {
 public:
  ReduceTask(const NetlevOptions& net, Host* host);
  ~ReduceTask();
  // before INIT: confine the task's files (merge service, foreign client)
  void set_sandbox(const TaskSandbox& sb) { sandbox_ = sb; }
  // before INIT: merge on this HIP device whatever mapred.uda.gpu.device says (a per-GPU node daemon)
  void set_forced_device(int d) { forced_device_ = d; }
  // Downcall from the host. Throws ProtocolError on a malformed/unsupported command.
  void handle(const HadoopCmd& cmd);
  // Close (reduceExitMsg): stop and join the merge thread.
  void exit();
  bool finished() const { return finished_.load(); }
  // attempt id from INIT ("" before INIT); read once the task has exited
  std::string task_id() const { return inited_ ? init_.reduce_task_id : std::string(); }
  ReduceStats stats() const;
  std::string stats_json() const;

  // exposed for the fetchers
  ClientTransport* transport() { return transport_.get(); }
  // Fetch [off, end) of a partition straight into dst + off (the RDMA-WRITE-into-the-reducer-buffer
  // analogue), `depth` requests of buffer_size_ in flight. Returns end.
  // Fetch [off, end) of a partition straight into dst with `depth` requests in flight. on_prefix(a, b):
  // bytes [a, b) have landed (called in order, each call after at least `prefix_step` new bytes, and
  // once more at the end, from a transport thread).
  int64_t fetch_direct(const FetchParams& f, uint8_t* dst, int64_t off, int64_t end, int depth,
                       const std::function<void(int64_t, int64_t)>& on_prefix = nullptr, int64_t prefix_step = 0);
  // in-flight fetch requests (exit() waits for their completions)
  void fetch_begin();
  void fetch_end();

 private:
  void on_init(const InitParams& p);
  void merge_main();
  void merge_online();
  void merge_hybrid();
  void merge_gpu();
  // Device fetch (descriptors, merge in place). probe: return false before consuming anything if the
  // first MOFs are not device-resident (the caller then runs merge_gpu()).
  bool merge_gpu_device(bool probe);
  // Device fetch: a partition the providers would not answer with a descriptor.
  struct DeclinedPart {
    FetchParams f;
    int64_t len = 0;
    std::string path;  // the MOF file the provider named, and the partition's offset in it
    int64_t file_off = 0;
  };
  // Their bytes into one device buffer (grown as needed; (*at)[k]: where partition k landed). Returns the
  // bytes fetched; *local: of those, read from the MOF files on this node.
  int64_t fetch_declined_bytes(int device, const std::vector<DeclinedPart>& parts, gpu::DeviceBuffer& dst,
                               std::vector<const uint8_t*>* at, int64_t* local);
  // Tell every provider in `hosts` that `holder` (this task) is done with its descriptors.
  void release_descriptors(const std::set<std::string>& hosts, const std::string& holder);
  // GPU backend: started at INIT on prewarm_thr_ (mapred.uda.gpu.prewarm): HIP context, SDMA engine,
  // code objects, a pooled workspace with its pinned D2H ring and early stager, pinned fetch-arena
  // blocks, all while the FETCHes are still to come (reduce slow-start). The merge joins it first.
  struct PrewarmConf {  // read on the INIT thread (the host's get_conf may be bound to it)
    bool early_h2d = true;
    int64_t pinned_bytes = 0;
    int64_t round_bytes = 2ll << 30;
    int maps = 0;
  };
  void prewarm_gpu(PrewarmConf pc);
  void join_prewarm();
  // GPU backend: the task's HIP device. mapred.uda.gpu.device = an index pins it; "auto" (default)
  // takes the visible GPU with the fewest live reduce tasks on the node (uda/node_registry.h), so a
  // node's reduce task processes spread over its GPUs. Registered until the task ends.
  // Runs once, on the prewarm thread (or the merge thread without prewarm): HIP's first call can
  // take a while in a fresh process and INIT must not wait for it.
  void place_on_gpu();
  std::once_flag placed_;
  TaskSandbox sandbox_;
  int forced_device_ = -1;
  std::string device_conf_ = "auto";   // read on the INIT thread
  std::string fault_spec_;             // mapred.uda.fault.inject (tests: faults of this task only)
  double hbm_budget_conf_ = 0;
  int device_ = 0;
  int registry_slot_ = -1;
  // Fetch `n` MOFs into `q` (reference merge_do_fetching_phase).
  void fetch_phase(MergeQueue* q, int n, std::vector<std::string>* map_ids = nullptr);
  // LPQ checkpoint (mapred.uda.lpq.checkpoint): completed LPQ spill files survive a failed attempt,
  // listed in a manifest keyed by job + partition; the next attempt skips their MOFs.
  void load_checkpoint();
  std::string checkpoint_path() const;
  void merging_phase(MergeQueue* q);
  std::unique_ptr<Segment> segment_for(std::shared_ptr<MofFetcher> f, int index);

  NetlevOptions net_;
  Host* host_;
  InitParams init_;
  KeyKind kind_ = KeyKind::kText;
  Codec codec_ = Codec::kNone;
  int64_t buffer_size_ = 0;        // per fetch buffer (pair = 2 of these)
  int64_t direct_chunk_ = 0;       // request size of fetch_direct (mapred.uda.fetch.request.bytes, >= buffer_size_)
  int64_t fetch_buf_ = 0;          // fetch chunk (== buffer_size_ uncompressed, the "rdma" half when compressed)
  int64_t kv_buf_size_ = 1 << 20;  // delivery buffer (NETLEV_KV_POOL_EXPO)
  int num_kv_bufs_ = 0;
  int num_lpqs_ = 0;
  int num_parallel_lpqs_ = 3;
  bool checkpoint_ = false;
  std::vector<std::string> restored_files_;   // LPQ files of the previous attempt, in LPQ order
  std::set<std::string> restored_maps_;       // their MOFs (FETCHes for these are dropped)
  std::map<std::string, std::string> restored_tasks_;  // map task -> attempt merged into a restored LPQ
  void discard_checkpoint();
  std::string backend_ = "cpu";
  std::unique_ptr<ClientTransport> transport_;

  // fetch bookkeeping
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<FetchParams> fetch_list_;
  int fetch_cmds_ = 0;  // FETCH commands received (restored ones included), under mu_
  std::deque<std::shared_ptr<MofFetcher>> fetched_;  // first chunk arrived
  int free_pairs_ = 0;
  int total_count_ = 0;
  int progress_count_ = 0;
  bool final_ = false;
  std::atomic<bool> stop_{false};
  std::atomic<bool> exiting_{false};  // exit() from the host (not a failure)
  std::atomic<bool> finished_{false};
  std::thread merge_thr_;
  std::thread prewarm_thr_;
  bool inited_ = false;
  int next_index_ = 0;

  std::mutex inflight_mu_;
  std::condition_variable inflight_cv_;
  int64_t inflight_ = 0;

  mutable std::mutex st_mu_;
  ReduceStats st_;
  friend class MofFetcher;
};

// Pulls one MOF partition chunk by chunk with one request in flight ahead of the consumer
// (double buffering, Segment::send_request in the reference); decompresses when a codec is set.
class MofFetcher : public std::enable_shared_from_this<MofFetcher> {
 public:
  MofFetcher(ReduceTask* task, FetchParams p, int64_t buf_size, Codec codec);
  void start();
  // ChunkSource: blocks until the next chunk is available; returns bytes (0 at end).
  int64_t pull(uint8_t* dst, int64_t cap);
  // GPU staging: copy the first chunk (the only one fetched so far) to dst and hand the buffer pair
  // back; the caller fetches the rest of the partition straight into its own memory.
  int64_t take_first(uint8_t* dst, int64_t cap);
  bool first_arrived() const { return first_done_; }
  const FetchParams& params() const { return p_; }
  int64_t part_len() const { return part_len_; }
  int64_t wait_ns = 0;

 private:
  // Prepare a fetch into buffer `buf` (mu_ held); the returned call runs after mu_ is released
  // because a transport may complete inline.
  std::function<void()> prepare(int buf);
  void on_done(int buf, const FetchAck& a);
  int64_t pull_raw(uint8_t* dst, int64_t cap);
  void release_pair();
  std::atomic<bool> released_{false};
  ReduceTask* task_;
  FetchParams p_;
  int64_t buf_size_;
  Codec codec_;
  std::unique_ptr<BlockDecoder> dec_;
  std::vector<uint8_t> bufs_[2];
  int64_t len_[2] = {0, 0};
  bool ready_[2] = {false, false};
  bool inflight_[2] = {false, false};
  int cur_ = 0;
  int64_t requested_ = 0;   // next offset to request
  int64_t consumed_ = 0;
  int64_t part_len_ = -1;
  FetchRequest proto_;
  bool first_done_ = false;
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace uda
