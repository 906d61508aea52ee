// Device shuffle/merge engine implementation. See device_engine.h for the design.
#include "device_engine.h"
#include "uda/fault.h"
#include "uda/trace.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <numeric>
#include <stdexcept>

#include "uda/log.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {
constexpr int kSlots = 2;  // recv/out double buffering across rounds


double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
}  // namespace

void hip_check(hipError_t e, const char* what, const char* file, int line) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " in " + what +
                             " at " + file + ":" + std::to_string(line));
}

// ------------------------------------------------------------------------------------ buffers
DeviceBuffer::~DeviceBuffer() { reset(); }
void DeviceBuffer::alloc(size_t bytes) {
  reset();
  if (bytes == 0) return;
  if (fault_hit("DEVICE_ALLOC")) throw std::runtime_error("injected device allocation failure");
  HIP_CHECK(hipMalloc(&ptr_, bytes));
  size_ = bytes;
}
void DeviceBuffer::reset() {
  if (ptr_) (void)hipFree(ptr_);
  ptr_ = nullptr;
  size_ = 0;
}

PinnedBuffer::~PinnedBuffer() {
  if (ptr_) (void)hipHostFree(ptr_);
}
PinnedPool& PinnedPool::instance() {
  static PinnedPool* pool = new PinnedPool();  // leaked on purpose: outlives every user at exit
  return *pool;
}

PinnedPool::Block PinnedPool::acquire(size_t min_bytes) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = free_.lower_bound(min_bytes);
    if (it != free_.end() && it->first <= 2 * min_bytes + PinnedArena::kBlock) {
      Block b{it->second, it->first};
      cached_ -= it->first;
      free_.erase(it);
      return b;
    }
  }
  Block b;
  b.size = (min_bytes + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
  void* p = nullptr;
  if (hipHostMalloc(&p, b.size, hipHostMallocDefault) != hipSuccess) {
    // trim the cache and retry once
    std::multimap<size_t, uint8_t*> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      drop.swap(free_);
      cached_ = 0;
    }
    for (auto& kv : drop) (void)hipHostFree(kv.second);
    if (hipHostMalloc(&p, b.size, hipHostMallocDefault) != hipSuccess)
      throw std::runtime_error("pinned host allocation of " + std::to_string(b.size) + " bytes failed");
  }
  b.p = static_cast<uint8_t*>(p);
  return b;
}

void PinnedPool::release(Block b) {
  if (!b.p) return;
  std::lock_guard<std::mutex> g(mu_);
  if (cached_ + b.size > cap_) {
    (void)hipHostFree(b.p);
    return;
  }
  free_.emplace(b.size, b.p);
  cached_ += b.size;
}

void PinnedPool::set_cache_cap(size_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  cap_ = bytes;
}

size_t PinnedPool::cached_bytes() {
  std::lock_guard<std::mutex> g(mu_);
  return cached_;
}

uint8_t* PinnedArena::alloc(size_t bytes) {
  bytes = (bytes + 255) & ~(size_t)255;
  bytes_ += bytes;
  if (bytes > kBlock / 4) {  // large request: a dedicated block, kept behind the shared one
    PinnedPool::Block b = PinnedPool::instance().acquire(std::max<size_t>(bytes, 256));
    if (last_shared_ && !blocks_.empty()) {
      blocks_.insert(blocks_.end() - 1, b);
    } else {
      blocks_.push_back(b);
      last_shared_ = false;
    }
    return b.p;
  }
  if (!last_shared_ || used_ + bytes > blocks_.back().size) {
    blocks_.push_back(PinnedPool::instance().acquire(kBlock));
    used_ = 0;
    last_shared_ = true;
  }
  uint8_t* p = blocks_.back().p + used_;
  used_ += bytes;
  return p;
}

void PinnedArena::release_all() {
  for (auto& b : blocks_) PinnedPool::instance().release(b);
  blocks_.clear();
  used_ = 0;
  last_shared_ = false;
  bytes_ = 0;
}

void PinnedBuffer::alloc(size_t bytes) {
  if (ptr_) (void)hipHostFree(ptr_);
  ptr_ = nullptr;
  size_ = 0;
  if (bytes == 0) return;
  HIP_CHECK(hipHostMalloc(&ptr_, bytes, hipHostMallocDefault));
  size_ = bytes;
}

std::string nccl_unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------------------ DeviceMerger
// Per-round plan blob layout (all int64 unless noted), uploaded with one H2D copy:
//   RunDesc runs[K] | int64 elem_off[K+1] | uint8_t* bases[K] | per pass p: seg_off, tile_prefix
DeviceMerger::DeviceMerger(int64_t max_records, int max_runs)
    : max_records_(max_records), max_runs_(max_runs) {
  elems_a_.alloc((size_t)std::max<int64_t>(max_records, 1) * sizeof(Elem));
  elems_b_.alloc((size_t)std::max<int64_t>(max_records, 1) * sizeof(Elem));
  // tiles per pass <= records/2048 + pairs; splits buffer sized for one pass
  const int64_t max_tiles = max_records / kMergeTile + max_runs + 2;
  splits_.alloc((size_t)max_tiles * sizeof(int64_t));
  flag_.alloc(sizeof(int));
  HIP_CHECK(hipMemset(flag_.as(), 0, sizeof(int)));
  int passes = 1;
  while ((1 << passes) < max_runs) ++passes;
  slot_bytes_ = (size_t)max_runs * (sizeof(RunDesc) + 2 * sizeof(int64_t) + sizeof(uint8_t*)) +
                (size_t)(passes + 1) * (2 * (max_runs + 2)) * sizeof(int64_t) + 256;
  slots_.resize(4);
  for (auto& s : slots_) {
    s.host.alloc(slot_bytes_);
    s.dev.alloc(slot_bytes_);
    HIP_CHECK(hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming));
  }
}

DeviceMerger::~DeviceMerger() {
  for (auto& s : slots_)
    if (s.uploaded) (void)hipEventDestroy(s.uploaded);
}

bool DeviceMerger::bad_layout() {
  int v = 0;
  HIP_CHECK(hipMemcpy(&v, flag_.as(), sizeof(int), hipMemcpyDeviceToHost));
  return v != 0;
}

int64_t DeviceMerger::merge_fixed(const std::vector<RunDesc>& runs, uint8_t* out, hipStream_t s) {
  const int K = (int)runs.size();
  if (K > max_runs_) throw std::runtime_error("DeviceMerger: too many runs");
  if (K > 65536) throw std::runtime_error("DeviceMerger: FIXED10 mode supports <= 65536 runs");
  int64_t total = 0;
  for (const auto& r : runs) total += r.nrec;
  if (total > max_records_) throw std::runtime_error("DeviceMerger: round exceeds capacity");
  last_passes_ = 0;
  if (total == 0) return 0;

  Slot& slot = slots_[next_slot_];
  next_slot_ = (next_slot_ + 1) % (int)slots_.size();
  if (slot.used) HIP_CHECK(hipEventSynchronize(slot.uploaded));
  slot.used = true;

  // ---- build the plan blob on the host
  uint8_t* h = slot.host.as();
  uint8_t* d = slot.dev.as();
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    size_t o = off;
    off = (size_t)align_up((int64_t)(off + bytes), 16);
    if (off > slot_bytes_) throw std::runtime_error("DeviceMerger: plan blob overflow");
    return o;
  };
  const size_t o_runs = carve(sizeof(RunDesc) * K);
  const size_t o_eoff = carve(sizeof(int64_t) * (K + 1));
  const size_t o_bases = carve(sizeof(uint8_t*) * K);
  std::memcpy(h + o_runs, runs.data(), sizeof(RunDesc) * K);
  int64_t* eoff = reinterpret_cast<int64_t*>(h + o_eoff);
  uint8_t** bases = reinterpret_cast<uint8_t**>(h + o_bases);
  eoff[0] = 0;
  for (int k = 0; k < K; ++k) {
    eoff[k + 1] = eoff[k] + runs[k].nrec;
    bases[k] = const_cast<uint8_t*>(runs[k].base);
  }
  // merge-tree passes over segment boundaries
  struct PassHost {
    size_t o_seg, o_tp;
    int nseg, npairs, ntiles;
  };
  std::vector<PassHost> passes;
  std::vector<int64_t> seg(eoff, eoff + K + 1);
  while ((int)seg.size() - 1 > 1) {
    const int S = (int)seg.size() - 1;
    const int P = (S + 1) / 2;
    PassHost ph;
    ph.nseg = S;
    ph.npairs = P;
    ph.o_seg = carve(sizeof(int64_t) * (S + 1));
    ph.o_tp = carve(sizeof(int64_t) * (P + 1));
    std::memcpy(h + ph.o_seg, seg.data(), sizeof(int64_t) * (S + 1));
    int64_t* tp = reinterpret_cast<int64_t*>(h + ph.o_tp);
    tp[0] = 0;
    std::vector<int64_t> next;
    next.push_back(0);
    for (int p = 0; p < P; ++p) {
      const int64_t beg = seg[2 * p];
      const int64_t end = seg[std::min(2 * p + 2, S)];
      tp[p + 1] = tp[p] + (end - beg + kMergeTile - 1) / kMergeTile;
      next.push_back(end);
    }
    ph.ntiles = (int)tp[P];
    passes.push_back(ph);
    seg.swap(next);
  }
  HIP_CHECK(hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipEventRecord(slot.uploaded, s));

  // ---- F2: keys
  Elem* cur = elems_a_.as<Elem>();
  Elem* nxt = elems_b_.as<Elem>();
  launch_extract_fixed(reinterpret_cast<const RunDesc*>(d + o_runs),
                       reinterpret_cast<const int64_t*>(d + o_eoff), K, total, cur,
                       flag_.as<int>(), s);
  // ---- F3: merge tree
  for (const auto& ph : passes) {
    PassDesc pd;
    pd.seg_off = reinterpret_cast<const int64_t*>(d + ph.o_seg);
    pd.tile_prefix = reinterpret_cast<const int64_t*>(d + ph.o_tp);
    pd.nseg = ph.nseg;
    pd.npairs = ph.npairs;
    pd.ntiles = ph.ntiles;
    launch_merge_partition(cur, pd, splits_.as<int64_t>(), s);
    launch_merge_pass(cur, nxt, pd, splits_.as<int64_t>(), s);
    std::swap(cur, nxt);
  }
  last_passes_ = (int)passes.size();
  // ---- F4: gather records into merged order
  launch_gather_fixed(cur, total, reinterpret_cast<uint8_t* const*>(d + o_bases), out, s);
  return total;
}

// -------------------------------------------------------------------------------- ShuffleJob
ShuffleJob::ShuffleJob(const ShuffleConfig& cfg) : cfg_(cfg) {
  if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world)
    throw std::runtime_error("ShuffleJob: bad rank/world");
  if (cfg_.maps_per_rank < 1) throw std::runtime_error("ShuffleJob: maps_per_rank < 1");
  if (cfg_.rounds < 1) cfg_.rounds = 1;
  if (cfg_.d2h_streams < 1) cfg_.d2h_streams = 1;
  HIP_CHECK(hipSetDevice(cfg_.device));
  int lo_prio = 0, hi_prio = 0;
  HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
  HIP_CHECK(hipStreamCreateWithPriority(&s_comm_, hipStreamNonBlocking, hi_prio));
  HIP_CHECK(hipStreamCreateWithFlags(&s_compute_, hipStreamNonBlocking));
  s_copy_.resize(cfg_.d2h_streams);
  for (auto& s : s_copy_) HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  buf_records_ = std::max<int64_t>(1, cfg_.kv_buf_bytes / kTeraRecordBytes);
  const int64_t buf_bytes = buf_records_ * kTeraRecordBytes;
  piece_bytes_ = std::max<int64_t>(1, cfg_.d2h_piece_bytes / buf_bytes) * buf_bytes;
  eof_buf_.alloc((size_t)buf_bytes + 16);
}

ShuffleJob::~ShuffleJob() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (copy_thr_.joinable()) copy_thr_.join();
  if (deliver_thr_.joinable()) deliver_thr_.join();
  (void)hipDeviceSynchronize();
  for (auto e : piece_events_) (void)hipEventDestroy(e);
  for (auto e : piece_start_ev_) (void)hipEventDestroy(e);
  for (auto e : out_free_ev_) (void)hipEventDestroy(e);
  for (auto e : join_ev_) (void)hipEventDestroy(e);
  for (auto& d : desc_slots_)
    if (d.uploaded) (void)hipEventDestroy(d.uploaded);
  exchange_.reset();
  for (auto s : s_copy_) (void)hipStreamDestroy(s);
  if (s_comm_) (void)hipStreamDestroy(s_comm_);
  if (s_compute_) (void)hipStreamDestroy(s_compute_);
}

void ShuffleJob::init_comm(const std::string& uid) {
  if (cfg_.world == 1) return;
  HIP_CHECK(hipSetDevice(cfg_.device));
  exchange_ = make_rccl_exchange(cfg_.rank, cfg_.world, uid);
}

void ShuffleJob::init_local() {
  if (cfg_.world == 1) return;
  if (cfg_.local_group.empty()) throw std::runtime_error("init_local: config.local_group is empty");
  HIP_CHECK(hipSetDevice(cfg_.device));
  exchange_ = make_local_exchange(cfg_.local_group, cfg_.rank, cfg_.world);
}

void ShuffleJob::generate() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  const int nruns = M * W;
  run_off_.assign(nruns, 0);
  run_nrec_.assign(nruns, 0);
  mof_off_.assign(M + 1, 0);
  int64_t off = 0;
  for (int m = 0; m < M; ++m) {
    mof_off_[m] = off;
    for (int d = 0; d < W; ++d) {
      const int64_t n = cfg_.records_per_map / W + (d < cfg_.records_per_map % W ? 1 : 0);
      run_nrec_[m * W + d] = n;
      run_off_[m * W + d] = off;
      off = align_up(off + n * kTeraRecordBytes + kEofBytes, 16);
    }
    off = align_up(off, 256);
  }
  mof_off_[M] = off;
  store_bytes_ = off;
  if (host_store()) {
    hstore_.alloc((size_t)store_bytes_);
    store_base_ = hstore_.as<uint8_t>();
    void* dp = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&dp, store_base_, 0));
    store_dev_base_ = reinterpret_cast<uint8_t*>(dp);
  } else if (cfg_.store == "hbm") {
    store_.alloc((size_t)store_bytes_);
    store_base_ = store_dev_base_ = store_.as<uint8_t>();
  } else {
    throw std::runtime_error("unknown store tier " + cfg_.store);
  }

  std::vector<uint8_t*> bases(nruns), gen_bases(nruns);
  std::vector<uint64_t> key_lo(nruns), key_span(nruns), seeds(nruns);
  const uint64_t step = (W == 1) ? ~0ull : (~0ull / (uint64_t)W);
  int64_t max_n = 0, max_mof = 0;
  DeviceBuffer tmp;  // host tier: one MOF at a time is generated in HBM, then copied out
  if (host_store()) {
    for (int m = 0; m < M; ++m) max_mof = std::max(max_mof, mof_off_[m + 1] - mof_off_[m]);
    tmp.alloc((size_t)max_mof);
  }
  for (int m = 0; m < M; ++m)
    for (int d = 0; d < W; ++d) {
      const int r = m * W + d;
      bases[r] = store_dev_base_ + run_off_[r];
      gen_bases[r] = host_store() ? tmp.as<uint8_t>() + (run_off_[r] - mof_off_[m]) : bases[r];
      key_lo[r] = step * (uint64_t)d;
      key_span[r] = step;
      const uint64_t gmap = (uint64_t)cfg_.rank * M + m;
      seeds[r] = cfg_.seed ^ (0x9E3779B97F4A7C15ull * (gmap + 1)) ^ (0xC2B2AE3D27D4EB4Full * (d + 1));
      max_n = std::max(max_n, run_nrec_[r]);
    }
  DeviceBuffer d_b(nruns * sizeof(uint8_t*)), d_n(nruns * 8), d_lo(nruns * 8), d_sp(nruns * 8),
      d_sd(nruns * 8), d_ck(nruns * 8);
  HIP_CHECK(hipMemcpy(d_b.as(), gen_bases.data(), nruns * sizeof(uint8_t*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_n.as(), run_nrec_.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_lo.as(), key_lo.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_sp.as(), key_span.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_sd.as(), seeds.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemset(d_ck.as(), 0, nruns * 8));
  if (!host_store()) {
    launch_teragen(d_b.as<uint8_t*>(), d_n.as<int64_t>(), d_lo.as<uint64_t>(), d_sp.as<uint64_t>(),
                   d_sd.as<uint64_t>(), nruns, max_n, d_ck.as<unsigned long long>(), s_compute_);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s_compute_));
  } else {
    for (int m = 0; m < M; ++m) {
      launch_teragen(d_b.as<uint8_t*>() + m * W, d_n.as<int64_t>() + m * W, d_lo.as<uint64_t>() + m * W,
                     d_sp.as<uint64_t>() + m * W, d_sd.as<uint64_t>() + m * W, W, max_n,
                     d_ck.as<unsigned long long>() + m * W, s_compute_);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(store_base_ + mof_off_[m], tmp.as(), (size_t)(mof_off_[m + 1] - mof_off_[m]),
                               hipMemcpyDeviceToHost, s_compute_));
    }
    HIP_CHECK(hipStreamSynchronize(s_compute_));
  }
  std::vector<uint64_t> ck(nruns);
  HIP_CHECK(hipMemcpy(ck.data(), d_ck.as(), nruns * 8, hipMemcpyDeviceToHost));
  dest_checksum_.assign(W, 0);
  dest_records_.assign(W, 0);
  for (int m = 0; m < M; ++m)
    for (int d = 0; d < W; ++d) {
      dest_checksum_[d] += ck[m * W + d];
      dest_records_[d] += run_nrec_[m * W + d];
    }
  // persistent per-run device tables for splitting
  d_run_bases_.alloc(nruns * sizeof(uint8_t*));
  d_run_nrec_.alloc(nruns * 8);
  d_bound_set_.alloc(nruns * sizeof(int));
  std::vector<int> bset(nruns);
  for (int r = 0; r < nruns; ++r) bset[r] = r % W;
  HIP_CHECK(hipMemcpy(d_run_bases_.as(), bases.data(), nruns * sizeof(uint8_t*), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_run_nrec_.as(), run_nrec_.data(), nruns * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_bound_set_.as(), bset.data(), nruns * sizeof(int), hipMemcpyHostToDevice));
  UDA_LOG(kInfo, "rank %d generated %d MOFs, %ld bytes in %s", cfg_.rank, M, (long)store_bytes_,
          host_store() ? "pinned host DRAM" : "HBM");
}

std::vector<int64_t> ShuffleJob::index_record(int m, int d) const {
  const int W = cfg_.world;
  if (m < 0 || m >= cfg_.maps_per_rank || d < 0 || d >= W) throw std::out_of_range("index_record");
  const int r = m * W + d;
  const int64_t part = run_nrec_[r] * kTeraRecordBytes + kEofBytes;
  return {run_off_[r] - mof_off_[m], part, part};
}

std::vector<uint8_t> ShuffleJob::read_partition(int m, int d) const {
  auto ir = index_record(m, d);
  std::vector<uint8_t> out((size_t)ir[2]);
  HIP_CHECK(hipMemcpy(out.data(), store_base_ + mof_off_[m] + ir[0], out.size(),
                      host_store() ? hipMemcpyHostToHost : hipMemcpyDeviceToHost));
  return out;
}

std::vector<std::vector<uint64_t>> ShuffleJob::sample_keys(int64_t every) {
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  const int nruns = M * W;
  every = std::max<int64_t>(1, every);
  std::vector<int64_t> soff(nruns + 1, 0);
  for (int r = 0; r < nruns; ++r) {
    const int64_t n = run_nrec_[r];
    const int64_t c = n > every / 2 ? (n - every / 2 + every - 1) / every : 0;
    soff[r + 1] = soff[r] + c;
  }
  const int64_t total = soff[nruns];
  std::vector<std::vector<uint64_t>> out(W);
  if (total == 0) return out;
  DeviceBuffer d_off((nruns + 1) * 8), d_out(total * sizeof(Elem));
  HIP_CHECK(hipMemcpy(d_off.as(), soff.data(), (nruns + 1) * 8, hipMemcpyHostToDevice));
  launch_sample_fixed(d_run_bases_.as<uint8_t*>(), d_run_nrec_.as<int64_t>(), nruns, every,
                      d_off.as<int64_t>(), total, d_out.as<Elem>(), s_compute_);
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  std::vector<Elem> h(total);
  HIP_CHECK(hipMemcpy(h.data(), d_out.as(), total * sizeof(Elem), hipMemcpyDeviceToHost));
  for (int r = 0; r < nruns; ++r) {
    auto& v = out[r % W];
    for (int64_t i = soff[r]; i < soff[r + 1]; ++i) {
      v.push_back(h[i].hi);
      v.push_back(h[i].lo);
    }
  }
  return out;
}

void ShuffleJob::set_bounds(const std::vector<uint64_t>& bounds) {
  const int W = cfg_.world, Q = cfg_.rounds;
  if ((int64_t)bounds.size() != (int64_t)W * (Q - 1) * 2)
    throw std::runtime_error("set_bounds: expected world*(rounds-1)*2 values");
  bounds_ = bounds;
  if (Q > 1) {
    d_bounds_.alloc(bounds.size() * 8);
    HIP_CHECK(hipMemcpy(d_bounds_.as(), bounds.data(), bounds.size() * 8, hipMemcpyHostToDevice));
  }
}

void ShuffleJob::compute_round_plans(std::vector<RoundPlan>* plans, double* ms) {
  const double t0 = now_ms();
  const int M = cfg_.maps_per_rank, W = cfg_.world, Q = cfg_.rounds;
  const int nruns = M * W;
  if (Q > 1 && bounds_.empty()) throw std::runtime_error("rounds > 1 requires set_bounds()");
  const int64_t per = Q + 1;
  if (d_split_out_.size() < (size_t)nruns * per * 8) d_split_out_.alloc((size_t)nruns * per * 8);
  launch_split_fixed(d_run_bases_.as<uint8_t*>(), d_run_nrec_.as<int64_t>(),
                     Q > 1 ? d_bounds_.as<Elem>() : nullptr, d_bound_set_.as<int>(), nruns, Q - 1,
                     d_split_out_.as<int64_t>(), s_compute_);
  std::vector<int64_t> pos((size_t)nruns * per);
  HIP_CHECK(hipMemcpyAsync(pos.data(), d_split_out_.as(), pos.size() * 8, hipMemcpyDeviceToHost,
                           s_compute_));
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  plans->assign(Q, RoundPlan());
  // send side and my-own counts; counts to exchange: [peer p][q][m]
  std::vector<int64_t> send_counts((size_t)W * Q * M), recv_counts((size_t)W * Q * M);
  for (int q = 0; q < Q; ++q) {
    auto& rp = (*plans)[q];
    rp.send_beg.assign((size_t)W * M, 0);
    rp.send_end.assign((size_t)W * M, 0);
    for (int p = 0; p < W; ++p)
      for (int m = 0; m < M; ++m) {
        const int r = m * W + p;
        rp.send_beg[p * M + m] = pos[(size_t)r * per + q];
        rp.send_end[p * M + m] = pos[(size_t)r * per + q + 1];
        send_counts[((size_t)p * Q + q) * M + m] = rp.send_end[p * M + m] - rp.send_beg[p * M + m];
      }
  }
  if (W == 1) {
    recv_counts = send_counts;
  } else {
    if (!exchange_) throw std::runtime_error("world > 1 requires init_comm() or init_local()");
    exchange_->alltoall_i64(send_counts.data(), recv_counts.data(), (size_t)Q * M, s_comm_);
  }
  for (int q = 0; q < Q; ++q) {
    auto& rp = (*plans)[q];
    rp.recv_cnt.assign((size_t)W * M, 0);
    rp.recv_records = 0;
    for (int s = 0; s < W; ++s)
      for (int j = 0; j < M; ++j) {
        const int64_t c = recv_counts[((size_t)s * Q + q) * M + j];
        rp.recv_cnt[s * M + j] = c;
        rp.recv_records += c;
      }
  }
  if (ms) *ms = now_ms() - t0;
}

void ShuffleJob::plan() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  compute_round_plans(&plans_, nullptr);
  max_round_records_ = 0;
  for (const auto& rp : plans_) max_round_records_ = std::max(max_round_records_, rp.recv_records);
  const int M = cfg_.maps_per_rank, W = cfg_.world;
  merger_.reset(new DeviceMerger(max_round_records_, M * W));
  const size_t slot_bytes = (size_t)std::max<int64_t>(1, max_round_records_) * kTeraRecordBytes;
  out_slots_.clear();
  recv_slots_.clear();
  out_slots_.resize(kSlots);
  for (auto& b : out_slots_) b.alloc(slot_bytes);
  if (W > 1 || host_store()) {
    recv_slots_.resize(kSlots);
    for (auto& b : recv_slots_) b.alloc(slot_bytes);
    desc_slots_.resize(4);
    for (auto& d : desc_slots_) {
      d.host.alloc(sizeof(CopyDesc) * (size_t)M * W + 64);
      d.dev.alloc(sizeof(CopyDesc) * (size_t)M * W + 64);
      HIP_CHECK(hipEventCreateWithFlags(&d.uploaded, hipEventDisableTiming));
    }
  }
  if (W > 1) {
    max_send_bytes_ = 0;
    for (const auto& rp : plans_) {
      int64_t sb = 0;
      for (int p = 0; p < W; ++p)
        if (p != cfg_.rank)
          for (int m = 0; m < M; ++m) sb += (rp.send_end[p * M + m] - rp.send_beg[p * M + m]) * kTeraRecordBytes;
      max_send_bytes_ = std::max(max_send_bytes_, sb);
    }
    pack_slots_.clear();
    pack_slots_.resize(kSlots);
    for (auto& b : pack_slots_) b.alloc((size_t)std::max<int64_t>(max_send_bytes_, 16));
  }
  d_validate_.alloc(256);
  if (cfg_.deliver_host && pinned_.size() == 0) {
    pinned_.alloc((size_t)piece_bytes_ * cfg_.pinned_slots);
    pinned_free_.assign(cfg_.pinned_slots, true);
    piece_events_.resize((size_t)cfg_.pinned_slots * cfg_.d2h_streams);
    piece_start_ev_.resize(cfg_.pinned_slots);
    for (auto& e : piece_events_) HIP_CHECK(hipEventCreate(&e));
    for (auto& e : piece_start_ev_) HIP_CHECK(hipEventCreate(&e));
    join_ev_.resize(cfg_.d2h_streams);
    for (auto& e : join_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    out_free_ev_.resize(kSlots);
    for (auto& e : out_free_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    copy_thr_ = std::thread([this] { copy_loop(); });
    deliver_thr_ = std::thread([this] { deliver_loop(); });
  }
  UDA_LOG(kInfo, "rank %d planned %d rounds, max round %ld records", cfg_.rank, cfg_.rounds,
          (long)max_round_records_);
}

// Copy thread: turns merged rounds into D2H pieces in the pinned ring (FIFO order).
void ShuffleJob::copy_loop() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int NS = (int)s_copy_.size();
  for (;;) {
    RoundOut r;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !round_q_.empty(); });
      if (stop_) return;
      r = round_q_.front();
      round_q_.pop_front();
    }
    for (auto s : s_copy_) HIP_CHECK(hipStreamWaitEvent(s, r.merged, 0));
    const int64_t total = r.records * kTeraRecordBytes;
    const bool last_round = (r.q == cfg_.rounds - 1);
    const uint8_t* src = out_slots_[r.out_slot].as<uint8_t>();
    int64_t off = 0;
    do {
      const int64_t len = std::min(piece_bytes_, total - off);
      int k = -1;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          if (stop_) return true;
          for (int i = 0; i < (int)pinned_free_.size(); ++i)
            if (pinned_free_[i]) return true;
          return false;
        });
        if (stop_) return;
        for (int i = 0; i < (int)pinned_free_.size(); ++i)
          if (pinned_free_[i]) {
            k = i;
            break;
          }
        pinned_free_[k] = false;
      }
      uint8_t* dst = pinned_.as<uint8_t>() + (int64_t)k * piece_bytes_;
      HIP_CHECK(hipEventRecord(piece_start_ev_[k], s_copy_[0]));
      // split the piece over the copy streams on whole-record boundaries
      const int64_t recs = len / kTeraRecordBytes;
      int64_t done = 0;
      // every copy stream starts the piece after the start event (stream 0); stream 0 then joins the
      // others, so piece_events_[k*NS] marks the whole piece and start->end is a same-stream interval
      for (int i = 0; i < NS; ++i) {
        const int64_t part = (i == NS - 1) ? (recs - done) : recs / NS;
        if (i > 0) HIP_CHECK(hipStreamWaitEvent(s_copy_[i], piece_start_ev_[k], 0));
        if (part > 0)
          HIP_CHECK(hipMemcpyAsync(dst + done * kTeraRecordBytes, src + off + done * kTeraRecordBytes,
                                   part * kTeraRecordBytes, hipMemcpyDeviceToHost, s_copy_[i]));
        if (i > 0) HIP_CHECK(hipEventRecord(piece_events_[(size_t)k * NS + i], s_copy_[i]));
        done += part;
      }
      for (int i = 1; i < NS; ++i) HIP_CHECK(hipStreamWaitEvent(s_copy_[0], piece_events_[(size_t)k * NS + i], 0));
      HIP_CHECK(hipEventRecord(piece_events_[(size_t)k * NS], s_copy_[0]));
      off += len;
      {
        std::lock_guard<std::mutex> g(mu_);
        piece_q_.push_back(Piece{k, len, last_round && off >= total, nullptr});
      }
      cv_.notify_all();
    } while (off < total);
    for (int i = 1; i < NS; ++i) {  // join the other copy streams before freeing the out slot
      HIP_CHECK(hipEventRecord(join_ev_[i], s_copy_[i]));
      HIP_CHECK(hipStreamWaitEvent(s_copy_[0], join_ev_[i], 0));
    }
    HIP_CHECK(hipEventRecord(out_free_ev_[r.out_slot], s_copy_[0]));
    {
      std::lock_guard<std::mutex> g(mu_);
      d2h_enqueued_[r.q] = 1;
    }
    cv_.notify_all();
  }
}

// Deliver thread: the "Java side" hand-off. Buffers hold whole records and are at most
// kv_buf_bytes; the final buffer carries the IFile EOF marker (-1,-1).
void ShuffleJob::deliver_loop() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int NS = (int)s_copy_.size();
  const int64_t buf_bytes = buf_records_ * kTeraRecordBytes;
  for (;;) {
    Piece p;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !piece_q_.empty(); });
      if (stop_) return;
      p = piece_q_.front();
      piece_q_.pop_front();
    }
    trace::Range tr_piece("uda.deliver_piece");
    HIP_CHECK(hipEventSynchronize(piece_events_[(size_t)p.slot * NS]));  // joins every copy stream
    float ms = 0;
    if (p.bytes > 0 && hipEventElapsedTime(&ms, piece_start_ev_[p.slot], piece_events_[(size_t)p.slot * NS]) == hipSuccess)
      step_d2h_ms_ += ms;
    const uint8_t* base = pinned_.as<uint8_t>() + (int64_t)p.slot * piece_bytes_;
    int err = 0;
    int64_t nb = 0;
    for (int64_t off = 0; off < p.bytes; off += buf_bytes) {
      const int64_t len = std::min(buf_bytes, p.bytes - off);
      const bool final_chunk = p.last && off + len >= p.bytes;
      if (final_chunk && len + kEofBytes <= cfg_.kv_buf_bytes) {
        uint8_t* e = eof_buf_.as<uint8_t>();
        std::memcpy(e, base + off, (size_t)len);
        e[len] = 0xFF;
        e[len + 1] = 0xFF;
        if (sink_ && !err) err = sink_(e, len + kEofBytes);
        ++nb;
        p.bytes = -1;  // EOF already delivered
        break;
      }
      if (sink_ && !err) err = sink_(base + off, len);
      ++nb;
    }
    if (p.last && p.bytes >= 0) {  // EOF did not fit (or empty final piece): separate buffer
      uint8_t* e = eof_buf_.as<uint8_t>();
      e[0] = 0xFF;
      e[1] = 0xFF;
      if (sink_ && !err) err = sink_(e, kEofBytes);
      ++nb;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      pinned_free_[p.slot] = true;
      step_buffers_ += nb;
      if (err) step_error_ = err;
      if (p.last) step_done_ = true;
    }
    cv_.notify_all();
  }
}

StepStats ShuffleJob::run_step() {
  trace::Range tr_step("uda.step");
  HIP_CHECK(hipSetDevice(cfg_.device));
  if (!merger_) throw std::runtime_error("run_step before plan()");
  StepStats st;
  const double t0 = now_ms();
  const int M = cfg_.maps_per_rank, W = cfg_.world, Q = cfg_.rounds, me = cfg_.rank;

  std::vector<RoundPlan> plans;
  compute_round_plans(&plans, &st.split_ms);
  for (int q = 0; q < Q; ++q)
    if (plans[q].recv_records > max_round_records_)
      throw std::runtime_error("round volume exceeds planned capacity");

  {
    std::lock_guard<std::mutex> g(mu_);
    d2h_enqueued_.assign(Q, 0);
    step_done_ = false;
    step_buffers_ = 0;
    step_error_ = 0;
    step_d2h_ms_ = 0;
  }
  std::vector<hipEvent_t> ev(4 * Q);
  for (auto& e : ev) HIP_CHECK(hipEventCreate(&e));
  std::vector<hipEvent_t> merged(kSlots), comm_done(kSlots);
  for (auto& e : merged) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : comm_done) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (cfg_.validate) HIP_CHECK(hipMemsetAsync(d_validate_.as(), 0, 256, s_compute_));
  unsigned long long* vstats = d_validate_.as<unsigned long long>();
  Elem* vprev = reinterpret_cast<Elem*>(d_validate_.as<uint8_t>() + 64);
  Elem* vlast = reinterpret_cast<Elem*>(d_validate_.as<uint8_t>() + 128);

  int64_t bytes_sent = 0;
  for (int q = 0; q < Q; ++q) {
    trace::Range tr_round("uda.round");
    const int slot = q % kSlots;
    const RoundPlan& rp = plans[q];
    std::vector<RunDesc> runs;
    if (W == 1 && !host_store()) {
      HIP_CHECK(hipEventRecord(ev[4 * q + 0], s_compute_));
      HIP_CHECK(hipEventRecord(ev[4 * q + 1], s_compute_));
      for (int m = 0; m < M; ++m) {
        RunDesc d;
        d.base = run_base(m, 0) + rp.send_beg[m] * kTeraRecordBytes;
        d.nrec = rp.send_end[m] - rp.send_beg[m];
        d.nbytes = d.nrec * kTeraRecordBytes;
        d.offsets = nullptr;
        runs.push_back(d);
      }
    } else {
      uint8_t* rbuf = recv_slots_[slot].as<uint8_t>();
      uint8_t* pbuf = W > 1 ? pack_slots_[slot].as<uint8_t>() : nullptr;
      if (q >= kSlots) HIP_CHECK(hipStreamWaitEvent(s_comm_, merged[slot], 0));
      HIP_CHECK(hipEventRecord(ev[4 * q + 0], s_comm_));
      std::vector<int64_t> roff((size_t)W * M + 1, 0);
      for (int i = 0; i < W * M; ++i) roff[i + 1] = roff[i] + rp.recv_cnt[i] * kTeraRecordBytes;
      // pack: per destination, this rank's slices of the round in map order, destinations in
      // rotating order; the self partition goes straight to its place in the receive slot
      DescSlot& ds = desc_slots_[next_desc_];
      next_desc_ = (next_desc_ + 1) % (int)desc_slots_.size();
      if (ds.used) HIP_CHECK(hipEventSynchronize(ds.uploaded));
      ds.used = true;
      CopyDesc* descs = ds.host.as<CopyDesc>();
      int nd = 0;
      int64_t max_bytes = 0;
      std::vector<int64_t> sb(W, 0), sd(W, 0), rb(W, 0), rd(W, 0);
      int64_t packed = 0;
      for (int k = 1; k < W; ++k) {
        const int to = (me + k) % W;
        sd[to] = packed;
        for (int m = 0; m < M; ++m) {
          const int64_t c = rp.send_end[to * M + m] - rp.send_beg[to * M + m];
          if (c <= 0) continue;
          descs[nd++] = CopyDesc{run_base(m, to) + rp.send_beg[to * M + m] * kTeraRecordBytes, pbuf + packed,
                                 c * kTeraRecordBytes};
          max_bytes = std::max(max_bytes, c * kTeraRecordBytes);
          packed += c * kTeraRecordBytes;
        }
        sb[to] = packed - sd[to];
      }
      for (int m = 0; m < M; ++m) {
        const int64_t c = rp.send_end[me * M + m] - rp.send_beg[me * M + m];
        if (c <= 0) continue;
        descs[nd++] = CopyDesc{run_base(m, me) + rp.send_beg[me * M + m] * kTeraRecordBytes, rbuf + roff[me * M + m],
                               c * kTeraRecordBytes};
        max_bytes = std::max(max_bytes, c * kTeraRecordBytes);
      }
      for (int s = 0; s < W; ++s) {
        if (s == me) continue;
        rd[s] = roff[s * M];
        rb[s] = roff[(s + 1) * M] - roff[s * M];
      }
      bytes_sent += packed;
      if (nd > 0 && !host_store()) {
        HIP_CHECK(hipMemcpyAsync(ds.dev.as(), descs, sizeof(CopyDesc) * nd, hipMemcpyHostToDevice, s_comm_));
        HIP_CHECK(hipEventRecord(ds.uploaded, s_comm_));
        launch_batched_copy(ds.dev.as<CopyDesc>(), nd, max_bytes, s_comm_);
      } else if (nd > 0) {
        // spill tier: the slices stream H2D over PCIe (SDMA) straight into the pack / receive slots
        for (int i = 0; i < nd; ++i)
          HIP_CHECK(hipMemcpyAsync(descs[i].dst, descs[i].src, (size_t)descs[i].bytes, hipMemcpyHostToDevice, s_comm_));
        HIP_CHECK(hipEventRecord(ds.uploaded, s_comm_));
        st.bytes_h2d += [&] {
          int64_t b = 0;
          for (int i = 0; i < nd; ++i) b += descs[i].bytes;
          return b;
        }();
      }
      if (W > 1) exchange_->alltoallv(pbuf, sb.data(), sd.data(), rbuf, rb.data(), rd.data(), s_comm_);
      HIP_CHECK(hipEventRecord(ev[4 * q + 1], s_comm_));
      HIP_CHECK(hipEventRecord(comm_done[slot], s_comm_));
      HIP_CHECK(hipStreamWaitEvent(s_compute_, comm_done[slot], 0));
      for (int i = 0; i < W * M; ++i) {
        RunDesc d;
        d.base = rbuf + roff[i];
        d.nrec = rp.recv_cnt[i];
        d.nbytes = d.nrec * kTeraRecordBytes;
        d.offsets = nullptr;
        runs.push_back(d);
      }
    }
    // output slot reuse: the D2H of round q-kSlots must be enqueued (and is then waited on)
    if (cfg_.deliver_host && q >= kSlots) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return d2h_enqueued_[q - kSlots] != 0 || step_error_ != 0; });
      lk.unlock();
      HIP_CHECK(hipStreamWaitEvent(s_compute_, out_free_ev_[slot], 0));
    }
    HIP_CHECK(hipEventRecord(ev[4 * q + 2], s_compute_));
    uint8_t* out = out_slots_[slot].as<uint8_t>();
    const int64_t n = merger_->merge_fixed(runs, out, s_compute_);
    HIP_CHECK(hipGetLastError());
    st.merge_passes = std::max(st.merge_passes, merger_->last_passes());
    if (cfg_.validate && n > 0) {
      launch_validate_fixed(out, n, vprev, q > 0 ? 1 : 0, vlast, vstats, s_compute_);
      HIP_CHECK(hipMemcpyAsync(vprev, vlast, sizeof(Elem), hipMemcpyDeviceToDevice, s_compute_));
    }
    HIP_CHECK(hipEventRecord(ev[4 * q + 3], s_compute_));
    HIP_CHECK(hipEventRecord(merged[slot], s_compute_));
    st.records += n;
    if (cfg_.deliver_host) {
      {
        std::lock_guard<std::mutex> g(mu_);
        round_q_.push_back(RoundOut{q, slot, n, merged[slot]});
      }
      cv_.notify_all();
    }
  }
  if (cfg_.deliver_host) {
    std::unique_lock<std::mutex> lk(mu_);
    while (!cv_.wait_for(lk, std::chrono::milliseconds(100), [&] { return step_done_; })) {
      if (exchange_) {  // a lost peer must fail the step, not hang it
        lk.unlock();
        exchange_->check();
        lk.lock();
      }
    }
  }
  if (exchange_) exchange_->wait(s_comm_);
  HIP_CHECK(hipStreamSynchronize(s_compute_));
  HIP_CHECK(hipStreamSynchronize(s_comm_));
  for (auto s : s_copy_) HIP_CHECK(hipStreamSynchronize(s));
  st.wall_ms = now_ms() - t0;
  for (int q = 0; q < Q; ++q) {
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, ev[4 * q + 0], ev[4 * q + 1]) == hipSuccess) st.comm_ms += a;
    if (hipEventElapsedTime(&b, ev[4 * q + 2], ev[4 * q + 3]) == hipSuccess) st.merge_ms += b;
  }
  for (auto e : ev) (void)hipEventDestroy(e);
  for (auto e : merged) (void)hipEventDestroy(e);
  for (auto e : comm_done) (void)hipEventDestroy(e);
  st.d2h_ms = step_d2h_ms_;
  st.bytes_in = st.records * kTeraRecordBytes;
  st.bytes_sent = bytes_sent;
  st.buffers = step_buffers_;
  if (cfg_.validate) {
    unsigned long long v[2];
    HIP_CHECK(hipMemcpy(v, vstats, sizeof(v), hipMemcpyDeviceToHost));
    st.order_errors = (int64_t)v[0];
    st.checksum = v[1];
  }
  st.bad_layout = merger_->bad_layout();
  if (step_error_) throw std::runtime_error("delivery sink reported error " + std::to_string(step_error_));
  return st;
}

}  // namespace gpu
}  // namespace uda
