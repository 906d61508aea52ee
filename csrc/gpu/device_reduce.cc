// Device merge-and-deliver of one reduce task over HBM-resident partitions. See device_reduce.h.
#include "device_reduce.h"

#include <unistd.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "block_decoder.h"
#include "device_engine.h"
#include "hbm_ledger.h"
#include "sdma.h"
#include "uda/error.h"
#include "uda/trace.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Stream {
  hipStream_t s = nullptr;
  Stream() { HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
  ~Stream() {
    if (s) (void)hipStreamDestroy(s);
  }
};

struct Events {
  hipEvent_t e[2] = {nullptr, nullptr};
  Events() {
    for (auto& x : e) HIP_CHECK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  }
  ~Events() {
    for (auto x : e)
      if (x) (void)hipEventDestroy(x);
  }
};

// Per-device pool of everything a reduce task's device merge allocates: hipFree synchronizes the
// whole device, so allocating and freeing per task made 16 concurrent tasks stall one another at
// every task end. Buffers only grow; a workspace whose task failed is dropped, not reused.
struct FixedWs {
  int64_t pool_key = 0;  // input bytes of the task that last used it (FixedWsPool::acquire)
  std::unique_ptr<DeviceMerger> merger;
  DeviceBuffer out[2];
  DeviceBuffer d_bases, d_nrec, d_soff, d_samp, d_bset, d_out, d_bounds, d_runs, flag;
  // streaming decode of block-compressed runs (device_reduce_fixed_blocks): the round inputs, the block
  // prefixes + first keys, and the per-round decode descriptors
  DeviceBuffer in[2], prefix, d_first, d_keys, d_descs[2];
  hipStream_t s = nullptr;
  hipStream_t ds = nullptr;  // streaming decode: round decodes and cuts, beside the merges on s
  hipEvent_t merged[2] = {nullptr, nullptr};
  FixedWs() {
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (auto& e : merged) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ~FixedWs() {
    if (s) (void)hipStreamSynchronize(s);
    if (ds) {
      (void)hipStreamSynchronize(ds);
      (void)hipStreamDestroy(ds);
    }
    for (auto e : merged)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
  static void ensure(DeviceBuffer& b, size_t bytes) {
    if (b.size() < bytes) b.alloc_local(bytes + bytes / 8);
  }
  // the bytes ensure(b, bytes) allocates
  static int64_t grow(const DeviceBuffer& b, int64_t bytes) { return (int64_t)b.size() >= bytes ? 0 : bytes + bytes / 8; }
  int64_t device_bytes() const {
    int64_t n = merger ? merger->device_bytes() : 0;
    for (const DeviceBuffer* b : {&out[0], &out[1], &d_bases, &d_nrec, &d_soff, &d_samp, &d_bset, &d_out, &d_bounds,
                                  &d_runs, &flag, &in[0], &in[1], &prefix, &d_first, &d_keys, &d_descs[0], &d_descs[1]})
      n += (int64_t)b->held();
    return n;
  }
};

class FixedWsPool {
 public:
  static FixedWsPool& get() {
    static FixedWsPool* p = [] {
      auto* q = new FixedWsPool;  // never destroyed: tasks may outlive static teardown
      HbmLedger::get().add_pool({[q](int d, int64_t want) { return q->trim(d, want); },
                                 [q](int d) { return q->idle(d); }});
      return q;
    }();
    return *p;
  }
  // free idle workspaces of `device`, largest first, until `want` bytes are freed
  int64_t trim(int device, int64_t want) {
    std::vector<std::unique_ptr<FixedWs>> drop;
    int64_t got = 0;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = free_[device];
      std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a->device_bytes() < b->device_bytes(); });
      while (!v.empty() && got < want) {
        got += v.back()->device_bytes();
        drop.push_back(std::move(v.back()));
        v.pop_back();
      }
    }
    if (!drop.empty()) {
      int cur = 0;
      HIP_CHECK(hipGetDevice(&cur));
      HIP_CHECK(hipSetDevice(device));
      drop.clear();
      HIP_CHECK(hipSetDevice(cur));
    }
    return got;
  }
  int64_t idle(int device) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t n = 0;
    for (const auto& w : free_[device]) n += w->device_bytes();
    return n;
  }
  // the idle workspace last used by the task most like this one (closest pool_key = input bytes; ties
  // to the larger; key < 0: any), as DevicePool::acquire_fit in gpu_merge.cc
  std::unique_ptr<FixedWs> acquire(int device, int64_t key = -1) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = free_[device];
      if (!v.empty()) {
        size_t best = v.size() - 1;
        if (key >= 0)
          for (size_t i = 0; i < v.size(); ++i) {
            const int64_t b = v[best]->pool_key, c = v[i]->pool_key;
            const int64_t db = b > key ? b - key : key - b, dc = c > key ? c - key : key - c;
            if (dc < db || (dc == db && v[i]->device_bytes() > v[best]->device_bytes())) best = i;
          }
        auto w = std::move(v[best]);
        v.erase(v.begin() + (long)best);
        if (key >= 0) w->pool_key = key;
        return w;
      }
    }
    auto w = std::make_unique<FixedWs>();
    if (key >= 0) w->pool_key = key;
    return w;
  }
  void release(int device, std::unique_ptr<FixedWs> w) {
    std::lock_guard<std::mutex> g(mu_);
    auto& v = free_[device];
    if (v.size() < 64) v.push_back(std::move(w));
  }

 private:
  std::mutex mu_;
  std::map<int, std::vector<std::unique_ptr<FixedWs>>> free_;
};

struct WsLease {
  int device;
  std::unique_ptr<FixedWs> w;
  bool clean = false;
  explicit WsLease(int d, int64_t key = -1) : device(d), w(FixedWsPool::get().acquire(d, key)) {}
  ~WsLease() {
    if (clean) FixedWsPool::get().release(device, std::move(w));
  }
};

// Pinned ring + completion signals borrowed from the device's shared SDMA engine.
struct Ring {
  SdmaEngine& eng;
  size_t bytes;
  uint8_t* p = nullptr;
  std::vector<hsa_signal_t> sig;
  Ring(SdmaEngine& e, size_t b, int slots) : eng(e), bytes(b) {
    p = static_cast<uint8_t*>(eng.acquire_ring(bytes));
    for (int i = 0; i < slots; ++i) sig.push_back(eng.make_signal());
  }
  ~Ring() {
    // copies still in flight (an exception mid-round) must land before the block is reused
    for (auto s : sig) {
      try {
        SdmaEngine::wait(s);
      } catch (...) {
      }
      eng.destroy_signal(s);
    }
    eng.release_ring(p, bytes);
  }
};
}  // namespace

int64_t fixed_round_ws_bytes(int64_t round_bytes, int runs) {
  // two output slots grown 1/8 past a round that may run ~10 % over the mean, plus the merger's
  // per-round plan tables (cell splits, samples: ~2 % of the round) and its upload slots
  const double slot = (double)round_bytes * 1.1 * 1.125;
  return (int64_t)(2 * slot + 0.02 * (double)round_bytes) + (int64_t)runs * 4096 + (16ll << 20);
}

void prewarm_device_reduce(const DeviceReduceConfig& cfg, int runs, int count) {
  HIP_CHECK(hipSetDevice(cfg.device));
  const int64_t rec = std::max<int64_t>(1, cfg.round_bytes / kTeraRecordBytes);
  const int64_t mr = rec + rec / 8;  // rounds run a little over their mean
  const int64_t buf_bytes = std::max<int64_t>(1, cfg.kv_buf_bytes / kTeraRecordBytes) * kTeraRecordBytes;
  const int64_t piece = std::max<int64_t>(1, cfg.piece_bytes / buf_bytes) * buf_bytes;
  const int S = std::max(2, cfg.pinned_slots);
  // `count` workspaces and rings held at once, so the pools keep that many for concurrent tasks
  std::vector<std::unique_ptr<WsLease>> leases;
  std::vector<std::unique_ptr<Ring>> rings;
  for (int i = 0; i < std::max(1, count); ++i) {
    leases.push_back(std::make_unique<WsLease>(cfg.device));
    FixedWs& ws = *leases.back()->w;
    if (!ws.merger || ws.merger->max_records() < mr || ws.merger->max_runs() < runs) ws.merger.reset(new DeviceMerger(mr, runs));
    rings.push_back(std::make_unique<Ring>(SdmaEngine::for_device(cfg.device), (size_t)piece * S, S));
  }
  rings.clear();  // back to the engine's cache
  for (auto& l : leases) l->clean = true;
}

bool runs_are_fixed10(const std::vector<RunDesc>& runs, hipStream_t s) {
  if (runs.empty()) return true;
  int64_t max_n = 0;
  for (const auto& r : runs) {
    if (r.nbytes != r.nrec * kTeraRecordBytes) return false;
    max_n = std::max(max_n, r.nrec);
  }
  int device = 0;
  HIP_CHECK(hipGetDevice(&device));
  WsLease lease(device);
  DeviceBuffer& d_runs = lease.w->d_runs;
  DeviceBuffer& flag = lease.w->flag;
  FixedWs::ensure(d_runs, runs.size() * sizeof(RunDesc));
  FixedWs::ensure(flag, sizeof(int));
  HIP_CHECK(hipMemcpyAsync(d_runs.as(), runs.data(), runs.size() * sizeof(RunDesc), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(flag.as(), 0, sizeof(int), s));
  for (size_t b = 0; b < runs.size(); b += 65535)
    launch_check_fixed(d_runs.as<RunDesc>() + b, (int)std::min<size_t>(65535, runs.size() - b), max_n, flag.as<int>(), s);
  HIP_CHECK(hipGetLastError());  // the launch itself
  int bad = 0;
  HIP_CHECK(hipMemcpyAsync(&bad, flag.as(), sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  lease.clean = true;
  return bad == 0;
}

DeviceReduceStats device_reduce_fixed(const DeviceReduceConfig& cfg, const std::vector<RunDesc>& runs,
                                      const std::function<int(const uint8_t*, int64_t)>& sink) {
  trace::Range tr("uda.device_reduce");
  HIP_CHECK(hipSetDevice(cfg.device));
  if (const hipError_t pending = hipGetLastError(); pending != hipSuccess)  // a failure before this call
    throw std::runtime_error(std::string("device reduce: HIP error pending on entry: ") + hipGetErrorString(pending));
  DeviceReduceStats st;
  const double t0 = now_ms();
  const int K = (int)runs.size();
  if (K > 65536) throw std::runtime_error("device reduce: more than 65536 runs");
  int64_t N = 0;
  for (const auto& r : runs) N += r.nrec;
  WsLease lease(cfg.device, N * kTeraRecordBytes);
  FixedWs& ws = *lease.w;
  hipStream_t s = ws.s;
  const int64_t buf_records = std::max<int64_t>(1, cfg.kv_buf_bytes / kTeraRecordBytes);
  const int64_t buf_bytes = buf_records * kTeraRecordBytes;
  const int64_t piece = std::max<int64_t>(1, cfg.piece_bytes / buf_bytes) * buf_bytes;
  std::vector<uint8_t> tail((size_t)cfg.kv_buf_bytes + 16);
  auto emit = [&](const uint8_t* p, int64_t len) {
    const double a = now_ms();
    if (sink(p, len) != 0) throw std::runtime_error("dataFromUda callback failed");
    st.sink_ms += now_ms() - a;
    st.buffers++;
  };
  if (N == 0) {
    tail[0] = tail[1] = 0xFF;
    emit(tail.data(), kEofBytes);
    lease.clean = true;
    return st;
  }

  // ---- HBM admission: the round size must fit the budget next to everything else on the node
  HbmLedger& led = HbmLedger::get();
  int64_t round_bytes = std::max<int64_t>(cfg.round_bytes, kTeraRecordBytes);
  const bool caller_reserved = led.bound() != nullptr && led.bound()->device() == cfg.device;
  std::unique_ptr<HbmLedger::Reservation> res;
  if (!caller_reserved) {
    auto need = [&](int64_t rb) {
      // what this task allocates beyond the workspace's buffers that are already large enough (a pooled
      // workspace's other buffers do not shrink what a grown one takes: alloc frees, then allocates anew)
      const int64_t r = std::min(rb, N * kTeraRecordBytes), slot = (int64_t)((double)r * 1.1);
      return FixedWs::grow(ws.out[0], slot) + FixedWs::grow(ws.out[1], slot) + (int64_t)(0.02 * (double)r) + (int64_t)K * 4096 +
             (16ll << 20);
    };
    const int64_t hr = led.headroom(cfg.device);
    while (round_bytes > (64ll << 20) && need(round_bytes) > hr) round_bytes /= 2;
    res = led.reserve(cfg.device, need(round_bytes), cfg.stop);
    st.hbm_wait_ms = res->wait_ms();
    st.hbm_reserved = res->granted();
  }
  st.round_bytes = round_bytes;
  // ---- round plan: key sample -> Q-1 bounds -> per-run split positions
  const int Q = (int)std::max<int64_t>(1, (N * kTeraRecordBytes + round_bytes - 1) / round_bytes);
  std::vector<int64_t> pos((size_t)K * (Q + 1), 0);
  {
    std::vector<uint8_t*> bases(K);
    std::vector<int64_t> nrec(K);
    for (int k = 0; k < K; ++k) {
      bases[k] = const_cast<uint8_t*>(runs[k].base);
      nrec[k] = runs[k].nrec;
      pos[(size_t)k * (Q + 1) + Q] = nrec[k];
    }
    if (Q > 1) {
      // enough samples for Q quantiles even on small inputs
      const int64_t every = std::max<int64_t>(1, std::min<int64_t>(cfg.sample_every, N / (64 * (int64_t)Q)));
      std::vector<int64_t> soff(K + 1, 0);
      for (int k = 0; k < K; ++k) {
        const int64_t n = nrec[k];
        soff[k + 1] = soff[k] + (n > every / 2 ? (n - every / 2 + every - 1) / every : 0);
      }
      const int64_t ns = soff[K];
      DeviceBuffer &d_bases = ws.d_bases, &d_nrec = ws.d_nrec, &d_soff = ws.d_soff, &d_samp = ws.d_samp,
                   &d_bset = ws.d_bset, &d_out = ws.d_out, &d_bounds = ws.d_bounds;
      FixedWs::ensure(d_bases, K * sizeof(uint8_t*));
      FixedWs::ensure(d_nrec, K * 8);
      FixedWs::ensure(d_soff, (K + 1) * 8);
      FixedWs::ensure(d_samp, (size_t)std::max<int64_t>(ns, 1) * sizeof(Elem));
      FixedWs::ensure(d_bset, K * sizeof(int));
      FixedWs::ensure(d_out, (size_t)K * (Q + 1) * 8);
      FixedWs::ensure(d_bounds, (size_t)(Q - 1) * sizeof(Elem));
      HIP_CHECK(hipMemcpyAsync(d_bases.as(), bases.data(), K * sizeof(uint8_t*), hipMemcpyHostToDevice, s));
      HIP_CHECK(hipMemcpyAsync(d_nrec.as(), nrec.data(), K * 8, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipMemcpyAsync(d_soff.as(), soff.data(), (K + 1) * 8, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipMemsetAsync(d_bset.as(), 0, K * sizeof(int), s));
      std::vector<Elem> samp((size_t)ns);
      if (ns > 0) {
        launch_sample_fixed(d_bases.as<uint8_t*>(), d_nrec.as<int64_t>(), K, every, d_soff.as<int64_t>(), ns,
                            d_samp.as<Elem>(), s);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(samp.data(), d_samp.as(), (size_t)ns * sizeof(Elem), hipMemcpyDeviceToHost, s));
      }
      HIP_CHECK(hipStreamSynchronize(s));
      std::sort(samp.begin(), samp.end(),
                [](const Elem& a, const Elem& b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); });
      std::vector<Elem> bounds((size_t)Q - 1, Elem{~0ull, ~0ull});
      for (int q = 1; q < Q && ns > 0; ++q) bounds[(size_t)q - 1] = samp[(size_t)std::min<int64_t>(ns - 1, ns * q / Q)];
      HIP_CHECK(hipMemcpyAsync(d_bounds.as(), bounds.data(), (size_t)(Q - 1) * sizeof(Elem), hipMemcpyHostToDevice, s));
      launch_split_fixed(d_bases.as<uint8_t*>(), d_nrec.as<int64_t>(), d_bounds.as<Elem>(), d_bset.as<int>(), K, Q - 1,
                         d_out.as<int64_t>(), s);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(pos.data(), d_out.as(), pos.size() * 8, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
    }
  }
  auto P = [&](int k, int q) { return pos[(size_t)k * (Q + 1) + q]; };
  int64_t max_round = 0;
  std::vector<int64_t> round_recs(Q, 0);
  for (int q = 0; q < Q; ++q) {
    for (int k = 0; k < K; ++k) round_recs[q] += P(k, q + 1) - P(k, q);
    max_round = std::max(max_round, round_recs[q]);
  }
  st.rounds = Q;
  static const bool trace_rounds = std::getenv("UDA_DEVICE_REDUCE_TRACE") != nullptr;  // tools: progress lines
  if (trace_rounds)
    std::fprintf(stderr, "[device_reduce pid %d] planned %d runs x %d rounds, %lld records, max round %lld\n", (int)getpid(),
                 K, Q, (long long)N, (long long)max_round);
  if (!ws.merger || ws.merger->max_records() < max_round || ws.merger->max_runs() < K) {
    const int64_t mr = std::max<int64_t>(max_round, ws.merger ? ws.merger->max_records() : 0);
    const int mk = std::max(K, ws.merger ? ws.merger->max_runs() : 0);
    ws.merger.reset();
    ws.merger.reset(new DeviceMerger(mr, mk));
  }
  DeviceMerger& merger = *ws.merger;
  DeviceBuffer* out = ws.out;
  for (int i = 0; i < 2; ++i) FixedWs::ensure(out[i], (size_t)std::max<int64_t>(max_round, 1) * kTeraRecordBytes);
  struct {
    hipEvent_t* e;
  } merged{ws.merged};
  const int S = std::max(2, cfg.pinned_slots);
  Ring ring(SdmaEngine::for_device(cfg.device), (size_t)piece * S, S);
  st.plan_ms = now_ms() - t0;

  auto enqueue_merge = [&](int q) {
    std::vector<RunDesc> rq(K);
    for (int k = 0; k < K; ++k) {
      rq[k].base = runs[k].base + P(k, q) * kTeraRecordBytes;
      rq[k].nrec = P(k, q + 1) - P(k, q);
      rq[k].nbytes = rq[k].nrec * kTeraRecordBytes;
      rq[k].offsets = nullptr;
    }
    merger.merge_fixed(rq, {0, K}, out[q % 2].as<uint8_t>(), s);
    HIP_CHECK(hipGetLastError());
    st.merge_passes = std::max(st.merge_passes, merger.last_passes());
    HIP_CHECK(hipEventRecord(merged.e[q % 2], s));
  };
  SdmaEngine& eng = ring.eng;
  auto deliver_round = [&](int q) {
    const uint8_t* src = out[q % 2].as<uint8_t>();
    const int64_t bytes = round_recs[q] * kTeraRecordBytes;
    const bool last_round = q == Q - 1;
    const int64_t np = (bytes + piece - 1) / piece;
    auto issue = [&](int64_t k) {
      const int64_t off = k * piece, len = std::min(piece, bytes - off);
      hsa_signal_t sg = ring.sig[(size_t)(k % S)];
      SdmaEngine::arm(sg, eng.parts((size_t)len, 1));
      eng.copy_d2h(ring.p + (k % S) * piece, src + off, (size_t)len, sg, 1);
    };
    for (int64_t k = 0; k < std::min<int64_t>(np, S); ++k) issue(k);
    bool eof_sent = false;
    for (int64_t k = 0; k < np; ++k) {
      const double a = now_ms();
      SdmaEngine::wait(ring.sig[(size_t)(k % S)]);
      st.d2h_wait_ms += now_ms() - a;
      const uint8_t* base = ring.p + (k % S) * piece;
      const int64_t plen = std::min(piece, bytes - k * piece);
      for (int64_t off = 0; off < plen; off += buf_bytes) {
        const int64_t len = std::min(buf_bytes, plen - off);
        const bool final_chunk = last_round && k == np - 1 && off + len >= plen;
        if (final_chunk && len + kEofBytes <= cfg.kv_buf_bytes) {
          std::memcpy(tail.data(), base + off, (size_t)len);
          tail[(size_t)len] = tail[(size_t)len + 1] = 0xFF;
          emit(tail.data(), len + kEofBytes);
          eof_sent = true;
        } else {
          emit(base + off, len);
        }
      }
      if (k + S < np) issue(k + S);
    }
    st.bytes += bytes;
    if (last_round && !eof_sent) {
      tail[0] = tail[1] = 0xFF;
      emit(tail.data(), kEofBytes);
    }
  };

  enqueue_merge(0);
  for (int q = 0; q < Q; ++q) {
    if (q + 1 < Q) enqueue_merge(q + 1);  // its slot held round q-1, delivered in the last iteration
    const double a = now_ms();
    HIP_CHECK(hipEventSynchronize(merged.e[q % 2]));
    st.merge_wait_ms += now_ms() - a;
    if (trace_rounds) std::fprintf(stderr, "[device_reduce pid %d] round %d merged\n", (int)getpid(), q);
    deliver_round(q);
    if (trace_rounds) std::fprintf(stderr, "[device_reduce pid %d] round %d delivered\n", (int)getpid(), q);
  }
  if (merger.bad_layout()) throw std::runtime_error("device reduce: non-TeraSort record in a FIXED10 run");
  st.records = N;
  HIP_CHECK(hipStreamSynchronize(s));
  lease.clean = true;
  return st;
}

}  // namespace gpu
}  // namespace uda

namespace uda {
namespace gpu {

namespace {
int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
bool key_less(const Elem& a, const Elem& b) { return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo); }
}  // namespace

// Streaming decode (F6 per key-range round) of block-compressed FIXED10 partitions.
//
// Reference: DecompressorWrapper decodes block by block into a cyclic buffer next to the merge, so a
// reducer never holds a partition's decoded bytes whole (src/Merger/DecompressorWrapper.cc:85-114,
// 168-197). Here the partitions stay compressed in HBM and each key-range round decodes only the
// blocks its key range covers:
//   1. prefix pass: every block's first 128 raw bytes (launch_block_decode with a clip) give the key of
//      the first record that starts in it (records are 104 bytes from the partition's start, so the
//      offset is known) -- a block first-key index, one wave per block, ~0.1 % of a full decode;
//   2. round bounds: quantiles of those keys; per round and partition, the blocks from the last one
//      whose first key is below the round's low bound to the first one whose first key reaches its
//      high bound hold every record of the range (boundary blocks are decoded by both neighbours);
//   3. per round: decode those blocks into one of two round input buffers (record starts 16-byte
//      aligned), cut each run to exactly the round's keys (split_fixed), merge into one of two output
//      slots, deliver as device_reduce_fixed does. Device memory: two round inputs + two round outputs.
DeviceReduceStats device_reduce_fixed_blocks(const DeviceReduceConfig& cfg, int codec, const BlockPlan& plan,
                                             const std::function<int(const uint8_t*, int64_t)>& sink,
                                             bool* streamed) {
  trace::Range tr("uda.device_reduce_blocks");
  *streamed = false;
  DeviceReduceStats st;
  HIP_CHECK(hipSetDevice(cfg.device));
  const double t0 = now_ms();
  const int K = (int)plan.raw_offset.size() - 1;
  const int64_t NB = (int64_t)plan.descs.size();
  if (K <= 0 || K > 65536) return st;
  // ---- streams: FIXED10 raw sizes (records + the 2-byte EOF), their blocks
  std::vector<int64_t> nrec(K), raw0(K), blk0(K + 1, NB);
  int64_t N = 0;
  for (int k = 0; k < K; ++k) {
    raw0[k] = plan.raw_offset[k];
    const int64_t raw = plan.raw_offset[k + 1] - plan.raw_offset[k];
    if (raw < kEofBytes || (raw - kEofBytes) % kTeraRecordBytes != 0) return st;  // not FIXED10
    nrec[k] = (raw - kEofBytes) / kTeraRecordBytes;
    N += nrec[k];
  }
  {
    // descriptors are in stream order with ascending dst: stream k's blocks are those with dst in
    // [raw_offset[k], raw_offset[k + 1])
    int64_t b = 0;
    for (int k = 0; k < K; ++k) {
      while (b < NB && plan.descs[(size_t)b].dst < plan.raw_offset[k]) ++b;
      blk0[k] = b;
    }
    blk0[K] = NB;
  }
  auto R = [&](int64_t b, int k) { return plan.descs[(size_t)b].dst - raw0[k]; };  // block's raw offset in its stream
  // ---- prefix pass: the block first-key index
  constexpr int64_t kSlot = 128;  // >= 103 bytes to the first record start + 13 bytes of record head and key
  WsLease lease(cfg.device, N * kTeraRecordBytes);
  FixedWs& ws = *lease.w;
  hipStream_t s = ws.s;
  std::vector<int32_t> first(NB, -1);
  std::vector<DecodeDesc> pd(plan.descs);
  for (int k = 0; k < K; ++k)
    for (int64_t b = blk0[k]; b < blk0[k + 1]; ++b) {
      const int64_t rel = R(b, k);
      const int64_t f = (kTeraRecordBytes - rel % kTeraRecordBytes) % kTeraRecordBytes;
      if (rel + f + kTeraRecordBytes <= nrec[k] * kTeraRecordBytes && f + kTeraKeyOffset + kTeraKeyBytes <= pd[(size_t)b].raw)
        first[(size_t)b] = (int32_t)f;
      pd[(size_t)b].dst = b * kSlot;
    }
  if (NB > 0) {
    FixedWs::ensure(ws.prefix, (size_t)NB * kSlot);
    FixedWs::ensure(ws.d_first, (size_t)NB * 4);
    FixedWs::ensure(ws.d_keys, (size_t)NB * sizeof(Elem));
    FixedWs::ensure(ws.d_descs[0], (size_t)NB * sizeof(DecodeDesc));
    FixedWs::ensure(ws.flag, 2 * sizeof(int));
    HIP_CHECK(hipMemcpyAsync(ws.d_descs[0].as(), pd.data(), (size_t)NB * sizeof(DecodeDesc), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(ws.d_first.as(), first.data(), (size_t)NB * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(ws.flag.as(), 0, 2 * sizeof(int), s));
    launch_block_decode(codec, nullptr, ws.prefix.as<uint8_t>(), ws.d_descs[0].as<DecodeDesc>(), (int)NB,
                        ws.flag.as<int>(), s, kSlot);
    launch_block_first_keys(ws.prefix.as<uint8_t>(), kSlot, ws.d_first.as<int32_t>(), (int)NB, ws.d_keys.as<Elem>(),
                            ws.flag.as<int>() + 1, s);
    HIP_CHECK(hipGetLastError());
  }
  std::vector<Elem> keys((size_t)NB);
  int flags[2] = {0, 0};
  if (NB > 0) {
    HIP_CHECK(hipMemcpyAsync(keys.data(), ws.d_keys.as(), (size_t)NB * sizeof(Elem), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(flags, ws.flag.as(), sizeof(flags), hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  if (flags[0]) throw UdaError("corrupt compressed block in a map output partition");
  if (flags[1]) {  // not TeraSort-shaped records: the caller decodes whole partitions (generic merge)
    lease.clean = true;
    return st;
  }
  // per stream: the blocks where a record starts, with its key (ascending in a sorted run)
  std::vector<std::vector<std::pair<int64_t, Elem>>> idx(K);
  std::vector<Elem> samp;
  for (int k = 0; k < K; ++k)
    for (int64_t b = blk0[k]; b < blk0[k + 1]; ++b)
      if (first[(size_t)b] >= 0) {
        if (!idx[k].empty() && key_less(keys[(size_t)b], idx[k].back().second)) {  // not a sorted run
          lease.clean = true;
          return st;
        }
        idx[k].emplace_back(b, keys[(size_t)b]);
        samp.push_back(keys[(size_t)b]);
      }
  std::sort(samp.begin(), samp.end(), key_less);
  *streamed = true;
  auto emit_eof_only = [&] {
    uint8_t eof[2] = {0xFF, 0xFF};
    if (sink(eof, kEofBytes) != 0) throw std::runtime_error("dataFromUda callback failed");
    st.buffers++;
  };
  if (N == 0) {
    emit_eof_only();
    lease.clean = true;
    return st;
  }
  // ---- rounds: bounds from the block keys, each round's block range and input layout per stream
  HbmLedger& led = HbmLedger::get();
  int64_t round_bytes = std::max<int64_t>(cfg.round_bytes, kTeraRecordBytes);
  struct Span {
    int64_t b0 = 0, b1 = -1;        // blocks [b0, b1]
    int64_t rec0 = 0, rec1 = 0;     // whole records inside, stream record indices
    int64_t in_off = 0;             // decoded byte R(b0) lands here in the round input
  };
  int Q = 1;
  std::vector<Elem> bounds;
  std::vector<std::vector<Span>> spans;
  std::vector<int64_t> in_bytes, in_recs;
  auto plan_rounds = [&](int64_t rb) {
    Q = (int)std::max<int64_t>(1, (N * kTeraRecordBytes + rb - 1) / rb);
    bounds.assign((size_t)std::max(0, Q - 1), Elem{0, 0});
    for (int q = 1; q < Q; ++q) bounds[(size_t)q - 1] = samp.empty() ? Elem{~0ull, ~0ull} : samp[samp.size() * (size_t)q / (size_t)Q];
    spans.assign((size_t)Q, std::vector<Span>((size_t)K));
    in_bytes.assign((size_t)Q, 0);
    in_recs.assign((size_t)Q, 0);
    for (int q = 0; q < Q; ++q) {
      int64_t cur = 0;
      for (int k = 0; k < K; ++k) {
        Span& sp = spans[(size_t)q][(size_t)k];
        if (nrec[k] == 0 || blk0[k] == blk0[k + 1]) continue;
        const auto& ix = idx[k];
        // b0: the last block starting a record with a key below the low bound (round 0: the first block)
        sp.b0 = blk0[k];
        if (q > 0) {
          const Elem lo = bounds[(size_t)q - 1];
          auto it = std::lower_bound(ix.begin(), ix.end(), lo, [](const std::pair<int64_t, Elem>& a, const Elem& v) {
            return key_less(a.second, v);
          });
          if (it != ix.begin()) sp.b0 = std::prev(it)->first;
        }
        // b1: the first block starting a record with a key at or above the high bound (last round: the last block)
        sp.b1 = blk0[k + 1] - 1;
        if (q + 1 < Q) {
          const Elem hi = bounds[(size_t)q];
          auto it = std::lower_bound(ix.begin(), ix.end(), hi, [](const std::pair<int64_t, Elem>& a, const Elem& v) {
            return key_less(a.second, v);
          });
          if (it != ix.end()) sp.b1 = it->first;
        }
        if (sp.b1 < sp.b0) sp.b1 = sp.b0;
        const int64_t r0 = R(sp.b0, k), r1 = R(sp.b1, k) + plan.descs[(size_t)sp.b1].raw;
        sp.rec0 = (r0 + kTeraRecordBytes - 1) / kTeraRecordBytes;
        sp.rec1 = std::min(r1 / kTeraRecordBytes, nrec[k]);
        if (sp.rec1 < sp.rec0) sp.rec1 = sp.rec0;
        const int64_t lead = sp.rec0 * kTeraRecordBytes - r0;  // partial record before the first whole one
        sp.in_off = align_up(cur + lead, 16) - lead;            // record starts 16-byte aligned
        cur = sp.in_off + (r1 - r0);
        in_recs[(size_t)q] += sp.rec1 - sp.rec0;
      }
      in_bytes[(size_t)q] = align_up(cur, 256);
    }
  };
  auto need = [&](int64_t rb) {
    plan_rounds(rb);
    int64_t mi = 0, mr = 0;
    for (int q = 0; q < Q; ++q) {
      mi = std::max(mi, in_bytes[(size_t)q]);
      mr = std::max(mr, in_recs[(size_t)q]);
    }
    const int64_t ob = std::max<int64_t>(mr, 1) * kTeraRecordBytes, db = std::max<int64_t>(NB, 1) * (int64_t)sizeof(DecodeDesc);
    return FixedWs::grow(ws.in[0], std::max<int64_t>(mi, 256)) + FixedWs::grow(ws.in[1], std::max<int64_t>(mi, 256)) +
           FixedWs::grow(ws.out[0], ob) + FixedWs::grow(ws.out[1], ob) + FixedWs::grow(ws.d_descs[0], db) + FixedWs::grow(ws.d_descs[1], db) +
           (int64_t)(0.02 * (double)ob) + (int64_t)K * 4096 + (16ll << 20);
  };
  std::unique_ptr<HbmLedger::Reservation> res;
  const bool caller_reserved = led.bound() != nullptr && led.bound()->device() == cfg.device;
  if (!caller_reserved) {
    const int64_t hr = led.headroom(cfg.device);
    while (round_bytes > (64ll << 20) && need(round_bytes) > hr) round_bytes /= 2;
    res = led.reserve(cfg.device, need(round_bytes), cfg.stop);
    st.hbm_wait_ms = res->wait_ms();
    st.hbm_reserved = res->granted();
  } else {
    plan_rounds(round_bytes);
  }
  st.round_bytes = round_bytes;
  int64_t max_in = 0, max_recs = 0;
  for (int q = 0; q < Q; ++q) {
    max_in = std::max(max_in, in_bytes[(size_t)q]);
    max_recs = std::max(max_recs, in_recs[(size_t)q]);
  }
  for (auto& b : ws.in) FixedWs::ensure(b, (size_t)std::max<int64_t>(max_in, 256));
  for (auto& b : ws.out) FixedWs::ensure(b, (size_t)std::max<int64_t>(max_recs, 1) * kTeraRecordBytes);
  for (auto& b : ws.d_descs) FixedWs::ensure(b, (size_t)std::max<int64_t>(NB, 1) * sizeof(DecodeDesc));
  FixedWs::ensure(ws.d_bases, 2 * (size_t)K * sizeof(uint8_t*));
  FixedWs::ensure(ws.d_nrec, 2 * (size_t)K * 8);
  FixedWs::ensure(ws.d_bset, (size_t)K * sizeof(int));
  FixedWs::ensure(ws.d_bounds, 2 * 2 * sizeof(Elem));
  FixedWs::ensure(ws.d_out, 2 * (size_t)K * 4 * 8);
  HIP_CHECK(hipMemsetAsync(ws.d_bset.as(), 0, (size_t)K * sizeof(int), s));
  if (!ws.merger || ws.merger->max_records() < max_recs || ws.merger->max_runs() < K) {
    const int64_t mr = std::max<int64_t>(max_recs, ws.merger ? ws.merger->max_records() : 0);
    const int mk = std::max(K, ws.merger ? ws.merger->max_runs() : 0);
    ws.merger.reset();
    ws.merger.reset(new DeviceMerger(mr, mk));
  }
  DeviceMerger& merger = *ws.merger;
  st.rounds = Q;
  const int64_t buf_records = std::max<int64_t>(1, cfg.kv_buf_bytes / kTeraRecordBytes);
  const int64_t buf_bytes = buf_records * kTeraRecordBytes;
  const int64_t piece = std::max<int64_t>(1, cfg.piece_bytes / buf_bytes) * buf_bytes;
  const int SL = std::max(2, cfg.pinned_slots);
  Ring ring(SdmaEngine::for_device(cfg.device), (size_t)piece * SL, SL);
  std::vector<uint8_t> tail((size_t)cfg.kv_buf_bytes + 16);
  auto emit = [&](const uint8_t* p, int64_t len) {
    const double a = now_ms();
    if (sink(p, len) != 0) throw std::runtime_error("dataFromUda callback failed");
    st.sink_ms += now_ms() - a;
    st.buffers++;
  };
  if (!ws.ds) HIP_CHECK(hipStreamCreateWithFlags(&ws.ds, hipStreamNonBlocking));
  // the prefix pass and this task's earlier use of the buffers (on s) come first
  hipEvent_t planned = nullptr;
  HIP_CHECK(hipEventCreateWithFlags(&planned, hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(planned, s));
  HIP_CHECK(hipStreamWaitEvent(ws.ds, planned, 0));
  HIP_CHECK(hipEventDestroy(planned));
  hipStream_t ds = ws.ds;
  st.plan_ms = now_ms() - t0;
  std::vector<int64_t> round_recs((size_t)Q, 0);
  int64_t decoded_blocks = 0;
  // ---- round q: decode its blocks, cut the runs to its key range, merge
  auto enqueue_round = [&](int q) {
    const int par = q & 1;
    uint8_t* in = ws.in[par].as<uint8_t>();
    std::vector<DecodeDesc> rd;
    std::vector<uint8_t*> bases((size_t)K, in);
    std::vector<int64_t> n((size_t)K, 0);
    for (int k = 0; k < K; ++k) {
      const Span& sp = spans[(size_t)q][(size_t)k];
      if (sp.b1 < sp.b0 || nrec[k] == 0) continue;
      const int64_t r0 = R(sp.b0, k);
      for (int64_t b = sp.b0; b <= sp.b1; ++b) {
        DecodeDesc d = plan.descs[(size_t)b];
        d.dst = sp.in_off + (R(b, k) - r0);
        rd.push_back(d);
      }
      bases[(size_t)k] = in + sp.in_off + (sp.rec0 * kTeraRecordBytes - r0);
      n[(size_t)k] = sp.rec1 - sp.rec0;
    }
    decoded_blocks += (int64_t)rd.size();
    struct Turn {
      const DeviceReduceConfig& c;
      bool held = false;
      ~Turn() {
        if (held && c.decode_done) c.decode_done();
      }
    } turn{cfg};
    if (cfg.decode_turn) {
      const double w = now_ms();
      if (!cfg.decode_turn()) throw UdaError("reduce task stopped while waiting for a device decode turn");
      turn.held = true;
      st.decode_wait_ms += now_ms() - w;
    }
    // the round input was last read by round q-2's merge (on s)
    if (q >= 2) HIP_CHECK(hipStreamWaitEvent(ds, ws.merged[par], 0));
    HIP_CHECK(hipMemcpyAsync(ws.d_descs[par].as(), rd.data(), rd.size() * sizeof(DecodeDesc), hipMemcpyHostToDevice, ds));
    launch_block_decode(codec, nullptr, in, ws.d_descs[par].as<DecodeDesc>(), (int)rd.size(), ws.flag.as<int>(), ds);
    // exactly the round's records of every run: [lower_bound(low), lower_bound(high))
    const Elem b2[2] = {q > 0 ? bounds[(size_t)q - 1] : Elem{0, 0}, q + 1 < Q ? bounds[(size_t)q] : Elem{~0ull, ~0ull}};
    uint8_t** dbases = ws.d_bases.as<uint8_t*>() + (size_t)par * K;
    int64_t* dn = ws.d_nrec.as<int64_t>() + (size_t)par * K;
    Elem* dbd = ws.d_bounds.as<Elem>() + 2 * par;
    int64_t* dpos = ws.d_out.as<int64_t>() + (size_t)par * K * 4;
    HIP_CHECK(hipMemcpyAsync(dbases, bases.data(), (size_t)K * sizeof(uint8_t*), hipMemcpyHostToDevice, ds));
    HIP_CHECK(hipMemcpyAsync(dn, n.data(), (size_t)K * 8, hipMemcpyHostToDevice, ds));
    HIP_CHECK(hipMemcpyAsync(dbd, b2, sizeof(b2), hipMemcpyHostToDevice, ds));
    launch_split_fixed(dbases, dn, dbd, ws.d_bset.as<int>(), K, 2, dpos, ds);
    HIP_CHECK(hipGetLastError());
    std::vector<int64_t> pos((size_t)K * 4);
    HIP_CHECK(hipMemcpyAsync(pos.data(), dpos, pos.size() * 8, hipMemcpyDeviceToHost, ds));
    HIP_CHECK(hipMemcpyAsync(flags, ws.flag.as(), sizeof(int), hipMemcpyDeviceToHost, ds));
    // the decode stream only: round q-1's merge keeps running on s (the merge of q follows it there)
    HIP_CHECK(hipStreamSynchronize(ds));
    if (flags[0]) throw UdaError("corrupt compressed block in a map output partition");
    std::vector<RunDesc> rq((size_t)K);
    int64_t total = 0;
    for (int k = 0; k < K; ++k) {
      const int64_t a = q > 0 ? pos[(size_t)k * 4 + 1] : 0;
      const int64_t e = q + 1 < Q ? pos[(size_t)k * 4 + 2] : n[(size_t)k];
      rq[(size_t)k].base = bases[(size_t)k] + a * kTeraRecordBytes;
      rq[(size_t)k].nrec = std::max<int64_t>(0, e - a);
      rq[(size_t)k].nbytes = rq[(size_t)k].nrec * kTeraRecordBytes;
      rq[(size_t)k].offsets = nullptr;
      total += rq[(size_t)k].nrec;
    }
    round_recs[(size_t)q] = total;
    merger.merge_fixed(rq, {0, K}, ws.out[par].as<uint8_t>(), s);
    HIP_CHECK(hipGetLastError());
    st.merge_passes = std::max(st.merge_passes, merger.last_passes());
    HIP_CHECK(hipEventRecord(ws.merged[par], s));
  };
  SdmaEngine& eng = ring.eng;
  bool eof_sent = false;
  auto deliver_round = [&](int q) {
    const uint8_t* src = ws.out[q & 1].as<uint8_t>();
    const int64_t bytes = round_recs[(size_t)q] * kTeraRecordBytes;
    const bool last_round = q == Q - 1;
    const int64_t np = (bytes + piece - 1) / piece;
    auto issue = [&](int64_t k) {
      const int64_t off = k * piece, len = std::min(piece, bytes - off);
      hsa_signal_t sg = ring.sig[(size_t)(k % SL)];
      SdmaEngine::arm(sg, eng.parts((size_t)len, 1));
      eng.copy_d2h(ring.p + (k % SL) * piece, src + off, (size_t)len, sg, 1);
    };
    for (int64_t k = 0; k < std::min<int64_t>(np, SL); ++k) issue(k);
    for (int64_t k = 0; k < np; ++k) {
      const double a = now_ms();
      SdmaEngine::wait(ring.sig[(size_t)(k % SL)]);
      st.d2h_wait_ms += now_ms() - a;
      const uint8_t* base = ring.p + (k % SL) * piece;
      const int64_t plen = std::min(piece, bytes - k * piece);
      for (int64_t off = 0; off < plen; off += buf_bytes) {
        const int64_t len = std::min(buf_bytes, plen - off);
        const bool final_chunk = last_round && k == np - 1 && off + len >= plen;
        if (final_chunk && len + kEofBytes <= cfg.kv_buf_bytes) {
          std::memcpy(tail.data(), base + off, (size_t)len);
          tail[(size_t)len] = tail[(size_t)len + 1] = 0xFF;
          emit(tail.data(), len + kEofBytes);
          eof_sent = true;
        } else {
          emit(base + off, len);
        }
      }
      if (k + SL < np) issue(k + SL);
    }
    st.bytes += bytes;
    if (last_round && !eof_sent) {
      tail[0] = tail[1] = 0xFF;
      emit(tail.data(), kEofBytes);
      eof_sent = true;
    }
  };
  // Rounds are delivered by a thread of their own, in order, while this one decodes, cuts and merges the
  // next: enqueue_round waits for its split positions (a stream sync that also covers the previous
  // round's merge), which in one thread held the round before it back from the link. Round q reuses
  // round q-2's slots, so it is enqueued once q-2 is delivered.
  std::mutex dmu;
  std::condition_variable dcv;
  int enqueued = 0, delivered = 0;
  bool abort = false;
  std::exception_ptr derr;
  std::thread dthr([&] {
    try {
      HIP_CHECK(hipSetDevice(cfg.device));
      for (int q = 0; q < Q; ++q) {
        {
          std::unique_lock<std::mutex> lk(dmu);
          dcv.wait(lk, [&] { return abort || enqueued > q; });
          if (abort) return;
        }
        const double a = now_ms();
        HIP_CHECK(hipEventSynchronize(ws.merged[q & 1]));
        st.merge_wait_ms += now_ms() - a;
        deliver_round(q);
        std::lock_guard<std::mutex> g(dmu);
        delivered = q + 1;
        dcv.notify_all();
      }
    } catch (...) {
      std::lock_guard<std::mutex> g(dmu);
      derr = std::current_exception();
      abort = true;
      dcv.notify_all();
    }
  });
  try {
    for (int q = 0; q < Q; ++q) {
      {
        std::unique_lock<std::mutex> lk(dmu);
        dcv.wait(lk, [&] { return abort || delivered >= q - 1; });
        if (abort) break;
      }
      enqueue_round(q);
      std::lock_guard<std::mutex> g(dmu);
      enqueued = q + 1;
      dcv.notify_all();
    }
  } catch (...) {
    {
      std::lock_guard<std::mutex> g(dmu);
      abort = true;
      dcv.notify_all();
    }
    dthr.join();
    throw;
  }
  dthr.join();
  if (derr) std::rethrow_exception(derr);
  if (merger.bad_layout()) throw std::runtime_error("device reduce: non-TeraSort record in a FIXED10 run");
  int64_t got = 0;
  for (int q = 0; q < Q; ++q) got += round_recs[(size_t)q];
  if (got != N)
    throw UdaError("streaming decode: the key-range rounds hold " + std::to_string(got) + " records, the partitions " +
                   std::to_string(N));
  st.records = N;
  st.decoded_blocks = decoded_blocks;
  HIP_CHECK(hipStreamSynchronize(ds));
  HIP_CHECK(hipStreamSynchronize(s));
  lease.clean = true;
  return st;
}

}  // namespace gpu
}  // namespace uda
