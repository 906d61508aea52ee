// Device-side shuffle + merge engine: the MI355X data path behind the Merger/MOFSupplier roles.
//
// Reference roles replaced:
//   * MOFSupplier DataEngine (src/MOFServer/IndexInfo.cc:141-376) reading MOF chunks from disk with
//     libaio and RDMA-writing them to reducers  ->  map-output partitions resident in HBM (or the
//     pinned-DRAM tier), shipped by an RCCL all-to-all over xGMI in key-range rounds.
//   * NetMerger MergeManager online merge (src/Merger/MergeManager.cc:47-193) with a CPU heap
//     k-way merge  ->  `DeviceMerger` (F2 keys, F3 merge-path tree, F4 gather) per round.
//   * merge_do_merging_phase -> dataFromUda (src/Merger/MergeManager.cc:155-182): merged records go
//     device -> host on the SDMA copy engines into a NUMA-local pinned ring and are handed to each
//     reduce task's consumer thread in <= kv_buf_size buffers of whole records, the last one
//     ending with the IFile EOF marker.
//
// Reduce tasks: every GPU hosts `reducers` reduce tasks (R); reducer i of GPU d owns the i-th
// contiguous slice of GPU d's key range (TotalOrderPartitioner semantics: the concatenation of all
// reducer outputs is globally sorted). Each reducer's range is cut into Q cells; cell (i, q) is
// shipped and merged in round q ("horizontal" rounds), so every round feeds all R consumers at
// once. Cell bounds come from a key sample taken when the job is planned (TeraSort's sampler).
//
// Pipeline per step (one process per GPU, W ranks):
//   comm stream    : [a2a round q+1] ...
//   compute stream : [extract + merge + gather round q (R independent groups)] ...
//   SDMA engines   : [D2H pieces of round q-1] ...   -> R consumer threads -> sink
// Round volumes are computed once in plan() (the map-side index records of the reference); a step
// only enqueues work and waits on the delivery handoff.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
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

#include "exchange.h"
#include "kernels.h"
#include "disk_store.h"
#include "sdma.h"

namespace uda {
namespace gpu {

void hip_check(hipError_t e, const char* what, const char* file, int line);
#define HIP_CHECK(x) ::uda::gpu::hip_check((x), #x, __FILE__, __LINE__)
// Throw if an earlier call on this thread left an error behind (kernel launches report theirs only
// through hipGetLastError): names the stretch of code it came from.
#define HIP_PENDING(where) ::uda::gpu::hip_check(hipGetLastError(), "a call before " where, __FILE__, __LINE__)

// Owning device allocation. Every allocation and free is accounted in the device's HBM ledger
// (hbm_ledger.h); `resident` marks data that stays (a map-output store), not a task's working set.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes, bool resident = false) { alloc(bytes, resident); }
  ~DeviceBuffer();
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept { take(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept {
    if (this != &o) {
      reset();
      take(o);
    }
    return *this;
  }
  // padded by ipc_safe_bytes(): another process may map the block over hipIpc
  void alloc(size_t bytes, bool resident = false) { alloc_impl(bytes, resident, true); }
  // a task's working set that never leaves this process: no hipIpc padding (a 2.3 GB round buffer
  // would otherwise hold 4.06 GB, past what its HBM reservation counted)
  void alloc_local(size_t bytes) { alloc_impl(bytes, false, false); }
  void reset();
  template <typename T = uint8_t>
  T* as() const {
    return reinterpret_cast<T*>(ptr_);
  }
  size_t size() const { return size_; }
  // bytes held in HBM (the allocation may be padded for hipIpc export)
  size_t held() const { return held_; }
  int device() const { return dev_; }

 private:
  void alloc_impl(size_t bytes, bool resident, bool exportable);
  void take(DeviceBuffer& o) {
    ptr_ = o.ptr_;
    size_ = o.size_;
    held_ = o.held_;
    dev_ = o.dev_;
    resident_ = o.resident_;
    guarded_ = o.guarded_;
    o.ptr_ = nullptr;
    o.size_ = o.held_ = 0;
    o.guarded_ = false;
  }
  void* ptr_ = nullptr;
  size_t size_ = 0;
  size_t held_ = 0;
  int dev_ = -1;
  bool resident_ = false;
  bool guarded_ = false;  // UDA_DEVICE_GUARD: the tail past size_ holds the guard pattern
};

// Owning pinned host allocation (pinned_host_alloc).
class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  ~PinnedBuffer();
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  PinnedBuffer(PinnedBuffer&& o) noexcept : ptr_(o.ptr_), size_(o.size_) {
    o.ptr_ = nullptr;
    o.size_ = 0;
  }
  void alloc(size_t bytes);
  // pinned pages placed on NUMA node `node` (< 0: anywhere)
  void alloc_on_node(size_t bytes, int node);
  template <typename T = uint8_t>
  T* as() const {
    return reinterpret_cast<T*>(ptr_);
  }
  size_t size() const { return size_; }

 private:
  void* ptr_ = nullptr;
  size_t size_ = 0;
};

// Process-wide cache of pinned host blocks (pinned_host_alloc). The GPU consumer stages fetched
// partitions and spill slices in them: page-locking / page-faulting and unmapping GBs per reduce
// task costs more than the merge itself, and a pinned source turns H2D into a direct DMA.
class PinnedPool {
 public:
  struct Block {
    uint8_t* p = nullptr;
    size_t size = 0;
  };
  static PinnedPool& instance();
  Block acquire(size_t min_bytes);
  void release(Block b);
  void set_cache_cap(size_t bytes);
  // Raise the cache cap to hold `bytes` (never lowers it), up to a quarter of the host memory this process
  // may use (physical memory, or its cgroup's limit). A task that pins its whole input each time (the
  // over-budget DRAM tier: 41.6 GB) otherwise re-pins what exceeds the default 32 GiB on every run.
  void raise_cache_cap(size_t bytes);
  size_t cached_bytes();
  // free every block the reaper has not freed yet, on this thread (before retrying a failed allocation)
  void drain_reaper();

 private:
  void reaper_main();
  std::mutex mu_;
  std::condition_variable reap_cv_;
  std::deque<Block> reap_;  // released past the cache cap: freed by the reaper thread
  bool reaper_started_ = false;
  int reaping_ = 0;
  std::multimap<size_t, uint8_t*> free_;
  size_t cached_ = 0;
  size_t cap_ = (size_t)32 << 30;
};

// Bump allocator over PinnedPool blocks; release_all() hands the blocks back to the pool.
class PinnedArena {
 public:
  static constexpr size_t kBlock = (size_t)256 << 20;
  PinnedArena() = default;
  ~PinnedArena() { release_all(); }
  PinnedArena(const PinnedArena&) = delete;
  PinnedArena& operator=(const PinnedArena&) = delete;
  uint8_t* alloc(size_t bytes);  // 256-byte aligned
  void release_all();
  size_t bytes() const { return bytes_; }

 private:
  std::vector<PinnedPool::Block> blocks_;
  size_t used_ = 0;   // bytes used in blocks_.back() (shared blocks only)
  bool last_shared_ = false;
  size_t bytes_ = 0;
};

// Merges K sorted FIXED10 runs on one stream. Enqueue-only: never synchronizes the host except
// when a plan slot is reused before its previous upload finished.
class DeviceMerger {
 public:
  DeviceMerger(int64_t max_records, int max_runs);
  ~DeviceMerger();
  // Merge `runs` (device-resident) into `out` (n*104 bytes). Runs are grouped: group g is runs
  // [group_first[g], group_first[g+1]) and merges into its own contiguous output range, groups in
  // order. Returns the record count.
  int64_t merge_fixed(const std::vector<RunDesc>& runs, const std::vector<int>& group_first, uint8_t* out,
                      hipStream_t s);
  // Number of merge-tree passes used by the last call.
  int last_passes() const { return last_passes_; }
  bool bad_layout();  // synchronizes; true if any record was not TeraSort-shaped
  int64_t max_records() const { return max_records_; }
  int max_runs() const { return max_runs_; }
  // HBM held by this merger's buffers
  int64_t device_bytes() const;
  // Cells the single-pass K-way merge handed to its wave-level PQ so far (synchronizes).
  int kway_overflow_cells();
  bool kway_enabled() const { return kway_; }

  // The single-pass K-way merge split in two: plan_kway enqueues a merge's cell planning on `s` into
  // one of two plan slots, run_kway its tiles (waiting for that plan on its own stream). A caller
  // can plan round q+1 on a side stream while round q's tiles run. kway_applicable: the runs can
  // take this path (at most kKwMaxRuns per group, within the merger's capacity).
  struct KwayPlan {
    KwayDesc kd;
    int64_t ncells = 0, total = 0;
    int pslot = 0;
  };
  bool kway_applicable(const std::vector<RunDesc>& runs, const std::vector<int>& group_first) const;
  KwayPlan plan_kway(const std::vector<RunDesc>& runs, const std::vector<int>& group_first, hipStream_t s);
  int64_t run_kway(const KwayPlan& p, uint8_t* out, hipStream_t s);

 private:
  int64_t merge_kway(const std::vector<RunDesc>& runs, const std::vector<int>& group_first, uint8_t* out,
                     hipStream_t s);
  struct Slot {
    PinnedBuffer host;
    DeviceBuffer dev;
    hipEvent_t uploaded = nullptr;
    bool used = false;
  };
  int64_t max_records_;
  int max_runs_;
  DeviceBuffer elems_a_, elems_b_, splits_;
  DeviceBuffer flag_;
  // single-pass K-way merge (kway.hip): samples (ping-pong), splitters, cell split table, overflow
  bool kway_ = true;
  int kw_cap_ = 2048;  // records per k-way cell (UDA_KWAY_CAP); in-place LDS merge: 4 workgroups per CU
  bool kw_staged_ = false;  // UDA_KWAY_STAGED: records staged in LDS once (kway_staged_kernel)
  DeviceBuffer kw_prof_, kw_overflow_;
  struct PlanBufs {  // per plan slot: samples, splitters, cell splits, sample-merge scratch
    DeviceBuffer samp_runs, samp_a, samp_b, bounds, split, splits;
    hipEvent_t planned = nullptr, used = nullptr;
    bool used_valid = false;
  };
  PlanBufs pbufs_[2];
  int next_pslot_ = 0;
  std::vector<Slot> slots_;
  int next_slot_ = 0;
  int last_passes_ = 0;
  size_t slot_bytes_ = 0;
};

// Delivery sink: called from reducer r's consumer thread with whole-record buffers
// (<= kv_buf_size). Return nonzero to abort the step.
using SinkFn = std::function<int(int reducer, const uint8_t* buf, int64_t len)>;

struct ShuffleConfig {
  int device = 0;
  int rank = 0;
  int world = 1;
  int maps_per_rank = 32;
  int64_t records_per_map = 1 << 20;
  int rounds = 8;                        // Q: cells per reducer
  int reducers = 1;                      // R: reduce tasks hosted by this GPU
  uint64_t seed = 0x5eed;
  int64_t kv_buf_bytes = 1 << 20;        // delivery buffer size (J2CQueue kv_buf_size)
  int64_t d2h_piece_bytes = 128ll << 20; // D2H granule (rounded down to whole buffers)
  int pinned_slots = 16;
  int d2h_engines = 1;                   // SDMA engines a piece is split over (if several are enabled)
  std::string d2h = "sdma";              // "sdma" (explicit copy engines) or "hip" (hipMemcpyAsync)
  bool deliver_host = true;              // false: stop after the device merge (ablation)
  bool validate = false;                 // device-side order/checksum/exchange checks every step
  std::string local_group;               // world > 1 without RCCL: ranks are threads of one process
  std::string store = "hbm";             // map-output store: "hbm", "host" (pinned DRAM) or "disk"
  std::string local_dirs;                // store=disk: comma-separated directories for the MOF files
  bool replan = false;                   // every step recomputes the cell splits and exchanges the counts
  bool map_sort = false;                 // setup: generate unsorted map input and sort it on the device (F8)
  // validate steps: also checksum every round's merged output right before its D2H (device) and as the
  // consumer threads receive it (host), per (round, reducer); costs a host hash of every record
  bool check_delivery = false;
};

struct StepStats {
  double wall_ms = 0;          // host wall time of the whole step
  double comm_ms = 0;          // sum of per-round exchange time (device events on the comm stream)
  double merge_ms = 0;         // sum of per-round merge time (device events on the compute stream)
  double d2h_ms = 0;           // host time the delivery copies were outstanding (summed per piece)
  double wait_out_ms = 0;      // host time the merge waited for a free output slot (D2H-bound)
  double plan_ms = 0;          // replan: cell splits + counts exchange inside the step
  double stage_ms = 0;         // spill tiers: host time of the staging thread's rounds (H2D / disk reads)
  int64_t bytes_in = 0;        // partition bytes delivered to this GPU's reducers (records only)
  int64_t records = 0;
  int64_t bytes_sent = 0;      // bytes this rank sent to peers (excl. self)
  int64_t bytes_h2d = 0;       // spill tier: bytes streamed host -> device
  int64_t buffers = 0;         // sink invocations
  int merge_passes = 0;
  bool validated = false;      // the checks below ran
  int64_t order_errors = -1;   // validate only
  uint64_t checksum = 0;       // validate only: sum of record hashes seen by the device
  int64_t exchange_errors = -1;  // validate only: received slices whose checksum differs from the sender's
  bool bad_layout = false;
  // validate only, per-round localisation of a checksum mismatch (all counts over the step's rounds):
  int64_t pre_merge_errors = -1;  // received slices that differed from the sender's right before the merge
  int64_t own_errors = -1;        // own cells (read in place or staged) that differ from their plan-time checksum
  int64_t merge_errors = -1;      // (round, reducer) outputs whose checksum differs from the sum of their inputs'
  int64_t pre_d2h_errors = -1;    // check_delivery: outputs that changed between the merge and their D2H
  int64_t delivery_errors = -1;   // check_delivery: outputs the consumer received differently from the merge
  std::string diag;               // the first mismatching (round, reducer) of each kind, "" when all agree
  std::vector<double> round_comm_ms, round_merge_ms;  // per round: exchange / merge span (device events)
};

class ShuffleJob {
 public:
  explicit ShuffleJob(const ShuffleConfig& cfg);
  ~ShuffleJob();

  const ShuffleConfig& config() const { return cfg_; }
  // RCCL bootstrap; `uid` is the ncclUniqueId produced by rank 0 (nccl_unique_id()).
  void init_comm(const std::string& uid);
  // Single-process rehearsal: ranks are threads sharing this device (config.local_group).
  void init_local();
  // One process per rank on one node (several may share a GPU): shared-memory control plane named
  // `name` (agreed by all ranks) + pull copies from the peers' HBM mapped over hipIpc. Collective.
  void init_ipc(const std::string& name);
  // Map phase stand-in: generate maps_per_rank TeraSort MOFs into the partition store.
  void generate();
  // Every `every`-th key of every local run, grouped by destination GPU:
  // result[d] = flat (hi, lo) pairs.
  std::vector<std::vector<uint64_t>> sample_keys(int64_t every);
  // bounds: world x (reducers*rounds - 1) x 2 u64 (hi, lo16<<48), ascending per destination GPU;
  // cell c = i*rounds + q of GPU d is [bound(d, c-1), bound(d, c)).
  void set_bounds(const std::vector<uint64_t>& bounds);
  // Compute the exact per-round volumes (cell splits + counts exchange), allocate the round buffers
  // and start the delivery threads. Collective when world > 1.
  void plan();
  void set_sink(SinkFn sink) { sink_ = std::move(sink); }
  // One shuffle+merge+deliver pass over the whole dataset. Collective when world > 1.
  // validate: run the device-side order / checksum / exchange checks in this step.
  StepStats run_step(bool validate);
  // The step's metadata again (cfg.replan): split every map output at the cell bounds and exchange
  // the per-slice counts, checked against the plan (the map outputs must not change between steps).
  void refresh_plan();

  // Per-destination-GPU checksum of locally generated records (sum of record_hash).
  std::vector<uint64_t> local_dest_checksums() const { return dest_checksum_; }
  std::vector<int64_t> local_dest_records() const { return dest_records_; }
  // Records each of this GPU's reducers receives per step (after plan()).
  std::vector<int64_t> reducer_records() const { return reducer_records_; }
  int64_t store_bytes() const { return store_bytes_; }
  double map_sort_ms() const { return map_sort_ms_; }  // cfg.map_sort: device time of the map-side sorts
  // Device address / size of MOF m in the partition store (host address for the host tier).
  const uint8_t* mof_device_ptr(int m) const { return store_dev_base_ + mof_off_.at(m); }
  // Drop the HBM store once its bytes live elsewhere (the API bench's compressed copy or MOF files);
  // the plan's metadata (index records, expected counts) stays valid, steps do not.
  void release_store() {
    store_.reset();
    store_base_ = store_dev_base_ = nullptr;
  }
  int64_t mof_bytes(int m) const { return mof_off_.at(m + 1) - mof_off_.at(m); }
  int64_t max_round_records() const { return max_round_records_; }
  // bytes this rank sends to each peer per step (self: 0)
  std::vector<int64_t> peer_send_bytes() const {
    std::vector<int64_t> v((size_t)cfg_.world, 0);
    for (const auto& rp : plans_)
      for (int p = 0; p < (int)rp.send.size() && p < cfg_.world; ++p)
        for (const auto& sp : rp.send[p]) v[(size_t)p] += sp.bytes;
    return v;
  }
  int comm_ranks() const { return exchange_ ? exchange_->comm_ranks() : 1; }
  std::string exchange_name() const { return exchange_ ? exchange_->name() : "none"; }
  std::string delivery_name() const;
  // Index record of (local map m, destination GPU d): offset, rawLength, partLength within MOF m.
  std::vector<int64_t> index_record(int m, int d) const;
  std::string store_name() const;
  // Copy a MOF partition (records + EOF) to host (tests / provider fallback path).
  std::vector<uint8_t> read_partition(int m, int d) const;

 private:
  struct RoundPlan {
    // send[p]: slices to GPU p, order (reducer i, local map m); empty for p == me
    std::vector<std::vector<Span>> send;
    int64_t send_bytes = 0;
    // recv_cnt[(s*R + i)*M + j]: records of source s's map j for my reducer i
    std::vector<int64_t> recv_cnt;
    std::vector<int64_t> recv_off;     // byte offset of that slice in the receive slot (s-major)
    std::vector<int64_t> self_beg;     // [i*M + m] first record of my own cell (i, q) in run (m, me)
    std::vector<int64_t> group_recs;   // records per reducer this round
    int64_t recv_records = 0;
    // spill tiers, world > 1: the outgoing slices are staged into HBM, one contiguous region per
    // peer (send staging of parity q & 1), and travel as one message per peer; the receive side
    // takes them as one span per source (its slices from a source are contiguous in the slot)
    std::vector<std::vector<Span>> staged_send, staged_recv;
  };
  void compute_plans();
  void copy_loop();
  void consume_loop(int reducer);
  void wait_exchange_ok();
  void localize_mismatch(StepStats& st);
  // Host-visible address of a run (device address for the HBM store, host address for the host
  // tier); kernels use the device-mapped addresses in d_run_bases_.
  uint8_t* run_base(int m, int d) const { return store_base_ + run_off_[m * cfg_.world + d]; }
  bool host_store() const { return cfg_.store == "host"; }
  bool disk_store() const { return cfg_.store == "disk"; }
  bool spilled() const { return host_store() || disk_store(); }  // own cells are staged, not read in place
  bool staged() const { return cfg_.world > 1 || spilled(); }
  // fn(r0, nr, bases, nrec, bound_set) over batches of runs whose records are device-readable: all
  // runs at once for the HBM / host stores, one MOF at a time (loaded from disk) for the disk store.
  void for_run_batches(const std::function<void(int, int, uint8_t* const*, const int64_t*, const int*)>& fn);

  ShuffleConfig cfg_;
  int R_ = 1, Q_ = 1, C_ = 1;  // reducers, rounds, cells (R*Q) per GPU
  std::unique_ptr<Exchange> exchange_;
  std::unique_ptr<DiskStore> disk_;
  hipStream_t s_comm_ = nullptr, s_compute_ = nullptr, s_copy_ = nullptr;
  hipStream_t s_plan_ = nullptr;  // K-way cell planning of the next round (runs read in place)
  DeviceBuffer store_;
  PinnedBuffer hstore_;
  uint8_t* store_base_ = nullptr;      // where run_base() points
  uint8_t* store_dev_base_ = nullptr;  // device-accessible alias for kernels
  int64_t store_bytes_ = 0;
  double map_sort_ms_ = 0;
  std::vector<int64_t> mof_off_, run_off_, run_nrec_;  // run index m*W + d
  std::vector<uint64_t> dest_checksum_;
  std::vector<uint64_t> run_gen_ck_;  // per run: the checksum its generation kernel computed
  std::vector<int64_t> dest_records_;
  std::vector<int64_t> reducer_records_;
  std::vector<uint64_t> bounds_;  // W x (C-1) x 2
  DeviceBuffer d_bounds_, d_run_bases_, d_run_nrec_, d_bound_set_, d_split_out_;
  std::vector<int64_t> split_pos_;  // [run r][cell c .. C]: (C+1) record positions per run
  std::vector<RoundPlan> plans_;
  int64_t max_round_records_ = 0;
  std::vector<DeviceBuffer> recv_slots_, out_slots_;
  // spill tiers, world > 1: outgoing slices of round q staged in send_staging_[q & 1] (per peer
  // contiguous); sent_ev_[q & 1] marks the exchange that reads them on the comm stream
  DeviceBuffer send_staging_[2];
  std::vector<hipEvent_t> merged_ev_, comm_ev_, sent_ev_;  // per slot
  int64_t xseq_ = 0;  // exchanges issued so far (Exchange sequence numbers)
  std::unique_ptr<DeviceMerger> merger_;
  DeviceBuffer d_validate_;  // stats[4] | prev key[R] | last key[R]
  // exchange verification (validate steps, world > 1): per round, the received peer slices and
  // the checksums their senders computed at plan()
  std::vector<DeviceBuffer> d_verify_runs_, d_verify_expect_;
  std::vector<int> verify_n_;
  std::vector<int64_t> verify_max_nrec_;
  DeviceBuffer d_verify_got_;
  // validate steps, per round: the own cells the merge reads (in place, or staged into the receive slot)
  // with their plan-time checksums, the expected checksum of every (round, reducer) output (the sum of
  // its input slices' plan-time checksums), and the device-side per-round results:
  //   diag[q * diag_stride() + {0,1,2,3}] = peer-slice mismatches before / after the merge, own-cell
  //   mismatches before / after; + 4 + i: the checksum of reducer i's merged output
  std::vector<DeviceBuffer> d_own_runs_, d_own_expect_;
  std::vector<int> own_n_;
  std::vector<int64_t> own_max_nrec_;
  std::vector<uint64_t> expect_group_ck_;  // [q * R + i]
  DeviceBuffer d_diag_;
  int diag_stride() const { return 4 + R_; }
  // check_delivery: per (round, reducer) checksum of the output slot right before its D2H (copy thread)
  // and of the bytes the consumer threads received
  std::vector<uint64_t> pre_d2h_ck_, delivered_ck_;
  bool step_check_delivery_ = false;
  DeviceBuffer d_d2h_runs_, d_d2h_ck_;
  // pinned-DRAM tier: per-round batched H2D copy descriptors (device), their count and largest size
  std::vector<DeviceBuffer> h2d_descs_;
  std::vector<int> h2d_n_;
  std::vector<int64_t> h2d_max_;
  int h2d_blocks_ = 2048;  // workgroups per descriptor (UDA_H2D_BLOCKS)
  bool sdma_h2d_ = true;   // pinned-DRAM tier, W == 1: stage on an SDMA engine (UDA_H2D_SDMA)
  hipStream_t s_stage_ = nullptr;  // disk tier, W == 1: H2D of the staging thread
  int64_t buf_records_ = 0;
  int64_t piece_bytes_ = 0;

  // ---- delivery: copy thread -> pinned ring (SDMA) -> per-reducer consumer threads
  std::unique_ptr<SdmaEngine> sdma_;
  uint8_t* ring_ = nullptr;          // pinned_slots x piece_bytes_
  std::string ring_numa_;            // where the ring's pages live (/proc/self/numa_maps)
  std::vector<hsa_signal_t> piece_sig_;
  std::vector<hipEvent_t> piece_ev_;
  struct RoundOut {
    int q;
    int slot;
    std::vector<int64_t> group_recs;
  };
  struct Item {
    int pslot;          // pinned slot, -1 for an EOF-only item
    int64_t bytes;
    bool last;          // this reducer's final data: append EOF
    double issued_ms;
    int q;              // round of the bytes (check_delivery)
  };
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<RoundOut> round_q_;
  std::vector<std::deque<Item>> items_;  // per reducer
  std::vector<bool> pinned_free_;
  std::vector<int> out_free_;  // per round: its output slot may be reused
  std::thread copy_thr_;
  std::vector<std::thread> consumers_;
  bool stop_ = false;
  int eof_count_ = 0;
  int64_t step_buffers_ = 0;
  int step_error_ = 0;
  std::string step_error_msg_;
  double step_d2h_ms_ = 0;
  SinkFn sink_;
  std::vector<std::unique_ptr<uint8_t[]>> eof_bufs_;  // per reducer: final chunk + EOF marker
};

// ncclUniqueId as bytes (rank 0 creates, others receive it out of band).
std::string nccl_unique_id();
int device_count();

// Streams of finished tasks, kept per (device, priority) for the next task on the current device:
// creating a stream costs milliseconds and concurrent creations serialize in the runtime (a wave of 15
// hosted tasks waited up to 106 ms for theirs). A stream handed back may still hold queued work; its
// next user orders behind it. prewarm_streams() fills the device's pool ahead of a first wave.
hipStream_t pooled_stream(int priority = 0);
// UDA_DEVICE_GUARD=1: device buffers freed so far whose guard tail a kernel overwrote
int64_t device_guard_violations();
void return_stream(hipStream_t s);
void prewarm_streams(int device, int n);

}  // namespace gpu
}  // namespace uda
