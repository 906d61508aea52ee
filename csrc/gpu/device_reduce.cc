// Device merge-and-deliver of one reduce task over HBM-resident partitions. See device_reduce.h.
#include "device_reduce.h"

#include <unistd.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>

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
  hipStream_t s = nullptr;
  hipEvent_t merged[2] = {nullptr, nullptr};
  FixedWs() {
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (auto& e : merged) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  ~FixedWs() {
    if (s) (void)hipStreamSynchronize(s);
    for (auto e : merged)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
  static void ensure(DeviceBuffer& b, size_t bytes) {
    if (b.size() < bytes) b.alloc(bytes + bytes / 8);
  }
  int64_t device_bytes() const {
    int64_t n = merger ? merger->device_bytes() : 0;
    for (const DeviceBuffer* b : {&out[0], &out[1], &d_bases, &d_nrec, &d_soff, &d_samp, &d_bset, &d_out, &d_bounds,
                                  &d_runs, &flag})
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

void prewarm_device_reduce(const DeviceReduceConfig& cfg, int runs) {
  HIP_CHECK(hipSetDevice(cfg.device));
  WsLease lease(cfg.device);
  FixedWs& ws = *lease.w;
  const int64_t rec = std::max<int64_t>(1, cfg.round_bytes / kTeraRecordBytes);
  const int64_t mr = rec + rec / 8;  // rounds run a little over their mean
  if (!ws.merger || ws.merger->max_records() < mr || ws.merger->max_runs() < runs) ws.merger.reset(new DeviceMerger(mr, runs));
  const int64_t buf_bytes = std::max<int64_t>(1, cfg.kv_buf_bytes / kTeraRecordBytes) * kTeraRecordBytes;
  const int64_t piece = std::max<int64_t>(1, cfg.piece_bytes / buf_bytes) * buf_bytes;
  const int S = std::max(2, cfg.pinned_slots);
  {
    Ring ring(SdmaEngine::for_device(cfg.device), (size_t)piece * S, S);  // back to the engine's cache
  }
  lease.clean = true;
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
      return std::max<int64_t>(0, fixed_round_ws_bytes(std::min(rb, N * kTeraRecordBytes), K) - ws.device_bytes());
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
