#include "generic_merger.h"
#include "merge_plan.h"

#include "uda/log.h"
#include "uda/trace.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace uda {
namespace gpu {

namespace {
// All passes' tables (pairs, then tile prefix, per pass) in one upload into a buffer the merger keeps:
// a DeviceBuffer per pass meant a hipMalloc and a device-synchronizing hipFree per pass of every merge,
// which stalled the work of concurrent merges (pipelined RPQ rounds, other reduce tasks).
std::vector<PassDesc> upload_passes(const std::vector<MergePassPlan>& plans, DeviceBuffer& buf, hipStream_t s) {
  std::vector<int64_t> all;
  std::vector<size_t> at;
  for (const MergePassPlan& mp : plans) {
    at.push_back(all.size());
    all.insert(all.end(), mp.pairs.begin(), mp.pairs.end());
    all.insert(all.end(), mp.tile_prefix.begin(), mp.tile_prefix.end());
  }
  std::vector<PassDesc> out;
  if (plans.empty()) return out;
  if (buf.size() < all.size() * 8) buf.alloc(all.size() * 8 + all.size() * 2 + 256);
  HIP_CHECK(hipMemcpyAsync(buf.as(), all.data(), all.size() * 8, hipMemcpyHostToDevice, s));
  for (size_t i = 0; i < plans.size(); ++i) {
    PassDesc pd;
    pd.pairs = buf.as<int64_t>() + at[i];
    pd.tile_prefix = pd.pairs + plans[i].pairs.size();
    pd.npairs = plans[i].npairs;
    pd.ntiles = plans[i].ntiles;
    out.push_back(pd);
  }
  return out;
}
}  // namespace

void GenericMerger::reserve(int64_t records, int runs) {
  if (records <= cap_records_ && runs <= cap_runs_) return;
  records = std::max<int64_t>(records, 1);
  const int64_t max_tiles = records / kGenericMergeTile + runs + 2;
  elems_a_.alloc_local((size_t)records * sizeof(Elem));
  elems_b_.alloc_local((size_t)records * sizeof(Elem));
  splits_.alloc_local((size_t)max_tiles * 8);
  sizes_.alloc_local((size_t)records * 8);
  out_off_.alloc_local((size_t)(std::max<int64_t>(records, runs) + 1) * 8);  // also holds elem_off (runs+1)
  scan_tmp_.alloc_local((size_t)scan_tmp_elems(records) * 8);
  side_.alloc_local((size_t)records * 24);  // keyptr(8) recptr(8) keylen(4) reclen(4)
  cap_records_ = records;
  cap_runs_ = std::max(runs, cap_runs_);
}

int64_t GenericMerger::workspace_bytes() const {
  int64_t b = 0;
  for (const DeviceBuffer* x : {&eoff_, &rounds_, &elems_a_, &elems_b_, &splits_, &sizes_, &out_off_, &scan_tmp_, &cuts_,
                                &offsets_, &tables_, &side_, &ck_, &f1ws_})
    b += (int64_t)x->size();
  for (const auto& k : gk_)
    for (const DeviceBuffer* x : {&k.tab, &k.samp, &k.sa, &k.sb, &k.bounds, &k.split, &k.hist, &k.flag}) b += (int64_t)x->size();
  return b;
}

GenericMerger::~GenericMerger() {
  for (hipEvent_t e : round_ev_) (void)hipEventDestroy(e);
}

// One level of the single-pass K-way merge (generic_kway.hip): runs in[off[k], off[k+1]) (sorted),
// merged into out. The regular sample of the runs is merged by a recursive level when it is large
// (it has the same shape: K sorted runs), else by the pairwise passes. Returns false if a cell
// exceeded its capacity (out is then incomplete). Synchronizes `s`.
bool GenericMerger::kway_level(int depth, const Elem* in, const std::vector<int64_t>& off, const int64_t* d_off,
                               const int64_t* d_ord_off, Elem* out, const GenericKeyCtx& ctx, hipStream_t s,
                               bool launch_cells, int64_t* cells) {
  const int K = (int)off.size() - 1;
  const int64_t total = off[K];
  const int64_t cap = generic_kway_cap(), T = cap / 2;
  const int64_t step = std::max<int64_t>(1, (cap - T) / (K + 2));  // a cell holds <= T + K * step <= cap
  std::vector<int64_t> soff(K + 1, 0);
  for (int k = 0; k < K; ++k) {
    const int64_t n = off[k + 1] - off[k];
    soff[k + 1] = soff[k] + (n > step / 2 ? (n - step / 2 + step - 1) / step : 0);
  }
  const int64_t ns = soff[K];
  // at least (K + 1) / 2 cells: with fewer, the sample rounding (up to K * step / 2 elements per
  // cell) could exceed the (K + 2) * step slack of the capacity bound
  const int64_t C = ns == 0 ? 1 : std::max<int64_t>({1, (total + T - 1) / T, (int64_t)(K + 1) / 2});
  if (cells) *cells = C;
  if (gk_.size() < 3) gk_.resize(3);  // depth <= 2; sized up front so `b` stays valid across recursion
  KwayBuffers& b = gk_[(size_t)depth];
  auto ensure = [](DeviceBuffer& x, size_t bytes) {
    if (x.size() < bytes) x.alloc_local(bytes + bytes / 8 + 64);
  };
  const size_t ns_b = sizeof(Elem) * (size_t)std::max<int64_t>(ns, 1);
  ensure(b.tab, 8 * (size_t)(K + 1));
  ensure(b.samp, ns_b);
  ensure(b.sa, ns_b);
  ensure(b.sb, ns_b);
  ensure(b.bounds, sizeof(Elem) * (size_t)std::max<int64_t>(C, 1));
  ensure(b.split, 8 * (size_t)K * (size_t)(C + 1));
  ensure(b.hist, sizeof(int) * (size_t)K * (size_t)C);
  ensure(b.flag, 64);
  int64_t* d_soff = b.tab.as<int64_t>();
  HIP_CHECK(hipMemcpyAsync(d_soff, soff.data(), 8 * (K + 1), hipMemcpyHostToDevice, s));
  const Elem* m = b.samp.as<Elem>();
  if (ns > 0) {
    launch_gk_sample(in, d_off, d_soff, K, step, ns, b.samp.as<Elem>(), s);
    bool done = false;
    const char* rv = std::getenv("UDA_GKWAY_RECURSE");  // tests force recursion on small inputs
    const int64_t recurse_at = rv && *rv ? std::max<int64_t>(1, std::atoll(rv)) : kGkRecurseSamples;
    if (ns > recurse_at && depth < 2) {
      done = kway_level(depth + 1, b.samp.as<Elem>(), soff, d_soff, d_ord_off, b.sa.as<Elem>(), ctx, s);
      if (done) m = b.sa.as<Elem>();
    }
    if (!done) {
      Elem* sbuf[2] = {b.sa.as<Elem>(), b.sb.as<Elem>()};
      int w = 0;
      for (const PassDesc& pd : upload_passes(plan_merge_passes(soff, {0, K}, kGenericMergeTile), b.passtab, s)) {
        launch_merge_partition_generic(m, pd, splits_.as<int64_t>(), ctx, s);
        launch_merge_pass_generic(m, sbuf[w], pd, splits_.as<int64_t>(), ctx, s);
        m = sbuf[w];
        w ^= 1;
      }
    }
    launch_gk_pick(m, ns, C, b.bounds.as<Elem>(), s);
  }
  launch_gk_split_hist(ctx, in, d_off, d_ord_off, m, ns, d_soff, step, K, b.bounds.as<Elem>(), C, b.hist.as<int>(),
                       b.split.as<int64_t>(), s);
  if (!launch_cells) return true;
  HIP_CHECK(hipMemsetAsync(b.flag.as(), 0, 4, s));
  launch_gk_cells(ctx, in, d_off, K, b.split.as<int64_t>(), C, 0, C, out, b.flag.as<int>(), s);
  int overflow = 0;
  HIP_CHECK(hipMemcpyAsync(&overflow, b.flag.as(), 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return overflow == 0;
}

GenericMergeResult GenericMerger::merge(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                                        int kind, uint8_t* out, int64_t out_cap, int64_t kv_buf, hipStream_t s,
                                        const RoundFn& on_round, int64_t round_bytes) {
  trace::Range tr("uda.generic_merge");
  // UDA_GM_PROFILE=1: synchronize after each phase and print the split (diagnostic only)
  static const bool prof = std::getenv("UDA_GM_PROFILE") != nullptr;
  auto tp0 = std::chrono::steady_clock::now();
  std::vector<std::pair<const char*, double>> phases;
  auto phase = [&](const char* name) {
    if (!prof) return;
    HIP_CHECK(hipStreamSynchronize(s));
    auto t = std::chrono::steady_clock::now();
    phases.push_back({name, std::chrono::duration<double, std::milli>(t - tp0).count()});
    tp0 = t;
  };
  GenericMergeResult res;
  const int K = (int)runs.size();
  if (K == 0) {
    res.cuts = {0};
    return res;
  }
  if (K > (1 << 20)) throw std::runtime_error("GenericMerger: too many runs");
  // ---- per-run tables: bases | nbytes | counts | rec_bytes | status | offsets pointers
  const size_t tb = (size_t)K * (8 * 5 + 8) + 256;
  if (tables_.size() < tb) tables_.alloc(tb);
  uint8_t* t = tables_.as<uint8_t>();
  auto* d_bases = reinterpret_cast<uint8_t**>(t);
  auto* d_nbytes = reinterpret_cast<int64_t*>(t + 8 * K);
  auto* d_counts = reinterpret_cast<int64_t*>(t + 16 * K);
  auto* d_recb = reinterpret_cast<int64_t*>(t + 24 * K);
  auto* d_offp = reinterpret_cast<int64_t**>(t + 32 * K);
  auto* d_status = reinterpret_cast<int*>(t + 40 * K);
  HIP_CHECK(hipMemcpyAsync(d_bases, runs.data(), 8 * K, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_nbytes, run_bytes.data(), 8 * K, hipMemcpyHostToDevice, s));
  // ---- F1 pass 1: chain walk per run with 4 KiB checkpoints
  const int64_t CH = f1_chunk_bytes();
  std::vector<int64_t> chunk_base(K + 1, 0);
  for (int k = 0; k < K; ++k) chunk_base[k + 1] = chunk_base[k] + (run_bytes[k] + CH - 1) / CH;
  const int64_t nchunks = chunk_base[K];
  std::vector<int32_t> chunk_run((size_t)std::max<int64_t>(nchunks, 1));
  for (int k = 0; k < K; ++k)
    for (int64_t c = chunk_base[k]; c < chunk_base[k + 1]; ++c) chunk_run[(size_t)c] = k;
  const size_t ckb = (size_t)(K + 1) * 8 + (size_t)(std::max<int64_t>(nchunks, 1) + 1) * (8 + 8 + 8 + 4) + 64;
  if (ck_.size() < ckb) ck_.alloc(ckb);
  int64_t* d_cbase = ck_.as<int64_t>();
  int64_t* d_ckstart = d_cbase + (K + 1);
  int64_t* d_ckcount = d_ckstart + std::max<int64_t>(nchunks, 1);
  int64_t* d_ckord = d_ckcount + std::max<int64_t>(nchunks, 1);
  int32_t* d_crun = reinterpret_cast<int32_t*>(d_ckord + std::max<int64_t>(nchunks, 1) + 1);  // scan writes n+1
  HIP_CHECK(hipMemcpyAsync(d_cbase, chunk_base.data(), 8 * (K + 1), hipMemcpyHostToDevice, s));
  if (nchunks > 0)
    HIP_CHECK(hipMemcpyAsync(d_crun, chunk_run.data(), 4 * (size_t)nchunks, hipMemcpyHostToDevice, s));
  static const bool prof_f1 = std::getenv("UDA_F1_PROFILE") != nullptr;
  static const bool serial_f1 = std::getenv("UDA_F1_SERIAL") != nullptr;
  if (serial_f1 || prof_f1) {
    DeviceBuffer d_prof;
    if (prof_f1) d_prof.alloc((size_t)K * 16);
    launch_f1_scan(d_bases, d_nbytes, K, d_cbase, d_ckstart, d_ckcount, d_counts, d_recb, d_status, s,
                   prof_f1 ? d_prof.as<uint64_t>() : nullptr);
    if (prof_f1) {
      std::vector<uint64_t> pr((size_t)K * 2);
      HIP_CHECK(hipMemcpyAsync(pr.data(), d_prof.as(), 16 * K, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      uint64_t a = 0, b = 0;
      for (int k = 0; k < K; ++k) {
        a += pr[2 * k];
        b += pr[2 * k + 1];
      }
      fprintf(stderr, "[F1 profile] runs=%d mean cycles per run: stage=%.0f walk=%.0f\n", K, (double)a / K,
              (double)b / K);
    }
  } else {
    // parallel form: chunk transfer functions composed per superchunk and per run
    const int64_t SC = f1_super_chunks();
    std::vector<int64_t> sup_base(K + 1, 0);
    for (int k = 0; k < K; ++k) sup_base[k + 1] = sup_base[k] + (chunk_base[k + 1] - chunk_base[k] + SC - 1) / SC;
    const int64_t nsup = sup_base[K];
    std::vector<int32_t> sup_run((size_t)std::max<int64_t>(nsup, 1));
    for (int k = 0; k < K; ++k)
      for (int64_t j = sup_base[k]; j < sup_base[k + 1]; ++j) sup_run[(size_t)j] = k;
    const size_t wsb = f1_parallel_workspace(nchunks, nsup) + (size_t)(K + 1) * 8 + (size_t)(nsup + 1) * 4 + 64;
    phase("f1_host_tables");
    if (f1ws_.size() < wsb) f1ws_.alloc(wsb);
    phase("f1_ws_alloc");
    uint8_t* ws = f1ws_.as<uint8_t>();
    auto* d_supbase = reinterpret_cast<int64_t*>(ws);
    auto* d_suprun = reinterpret_cast<int32_t*>(ws + (size_t)(K + 1) * 8);
    uint8_t* d_fws = ws + (((size_t)(K + 1) * 8 + (size_t)(nsup + 1) * 4 + 255) & ~(size_t)255);
    HIP_CHECK(hipMemcpyAsync(d_supbase, sup_base.data(), 8 * (K + 1), hipMemcpyHostToDevice, s));
    if (nsup > 0) HIP_CHECK(hipMemcpyAsync(d_suprun, sup_run.data(), 4 * (size_t)nsup, hipMemcpyHostToDevice, s));
    launch_f1_parallel(d_bases, d_nbytes, K, d_cbase, d_crun, nchunks, d_supbase, d_suprun, nsup, d_fws, d_ckstart,
                       d_ckcount, d_counts, d_recb, d_status, s, kind);
    std::vector<int> st(K);
    HIP_CHECK(hipMemcpyAsync(st.data(), d_status, 4 * K, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    phase("f1_parallel");
    std::vector<int> redo;
    for (int k = 0; k < K; ++k)
      if (st[k] == 2) redo.push_back(k);
    if (!redo.empty()) {  // records longer than the entry table straddle chunks: serial walk
      DeviceBuffer d_redo(redo.size() * 4);
      HIP_CHECK(hipMemcpyAsync(d_redo.as(), redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
      launch_f1_scan(d_bases, d_nbytes, (int)redo.size(), d_cbase, d_ckstart, d_ckcount, d_counts, d_recb, d_status,
                     s, nullptr, d_redo.as<int>());
      HIP_CHECK(hipStreamSynchronize(s));
    }
    f1_serial_runs_ = (int)redo.size();
  }
  std::vector<int64_t> counts(K), recb(K);
  std::vector<int> status(K);
  HIP_CHECK(hipMemcpyAsync(counts.data(), d_counts, 8 * K, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(recb.data(), d_recb, 8 * K, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(status.data(), d_status, 4 * K, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int64_t> eoff(K + 1, 0);
  int64_t bytes = 0;
  for (int k = 0; k < K; ++k) {
    if (status[k] != 0) throw std::runtime_error("GenericMerger: corrupt or truncated IFile run " + std::to_string(k));
    eoff[k + 1] = eoff[k] + counts[k];
    bytes += recb[k];
  }
  const int64_t total = eoff[K];
  if (bytes > out_cap) throw std::runtime_error("GenericMerger: output capacity too small");
  res.records = total;
  res.bytes = bytes;
  phase("f1_scan");
  reserve(std::max(total, nchunks), K);
  phase("reserve");
  // offsets storage: run k gets counts[k]+1 entries
  const int64_t off_elems = total + K;
  if (offsets_.size() < (size_t)off_elems * 8) offsets_.alloc((size_t)off_elems * 8);
  std::vector<int64_t*> offp(K);
  for (int k = 0; k < K; ++k) offp[k] = offsets_.as<int64_t>() + eoff[k] + k;
  HIP_CHECK(hipMemcpyAsync(d_offp, offp.data(), 8 * K, hipMemcpyHostToDevice, s));
  // ---- F1 pass 2: every chunk re-walked in parallel from its checkpoint
  if (eoff_.size() < (size_t)(K + 1) * 8) eoff_.alloc((size_t)(K + 1) * 8);
  int64_t* d_eoff = eoff_.as<int64_t>();
  HIP_CHECK(hipMemcpyAsync(d_eoff, eoff.data(), 8 * (K + 1), hipMemcpyHostToDevice, s));
  for (int k = 0; k < K; ++k)  // empty runs have no chunk to write their terminating offset
    if (run_bytes[k] == 0) HIP_CHECK(hipMemsetAsync(offp[k], 0, 8, s));
  if (nchunks > 0) {
    launch_exclusive_scan(d_ckcount, d_ckord, nchunks, scan_tmp_.as<int64_t>(), s);
    launch_f1_index(d_bases, d_nbytes, d_cbase, d_crun, d_ckstart, d_ckcount, d_ckord, d_eoff, d_recb, d_offp,
                    nchunks, s);
  }
  phase("f1_index");
  GenericKeyCtx ctx;
  ctx.bases = d_bases;
  ctx.offsets = const_cast<const int64_t* const*>(d_offp);
  ctx.kind = kind;
  {
    const int64_t nrec = std::max<int64_t>(total, 1);
    ctx.keyptr = reinterpret_cast<const uint8_t**>(side_.as<uint8_t>());
    ctx.recptr = reinterpret_cast<const uint8_t**>(side_.as<uint8_t>() + 8 * nrec);
    ctx.keylen = reinterpret_cast<int32_t*>(side_.as<uint8_t>() + 16 * nrec);
    ctx.reclen = reinterpret_cast<int32_t*>(side_.as<uint8_t>() + 20 * nrec);
  }
  if (total == 0) {
    res.cuts = {0};
    return res;
  }
  // ---- F2: normalize
  Elem* cur = elems_a_.as<Elem>();
  Elem* nxt = elems_b_.as<Elem>();
  launch_normalize_generic(ctx, d_eoff, K, total, cur, s);
  phase("f2_normalize");
  // ---- F3: single-pass K-way merge (generic_kway.hip) when K allows, else the pairwise tree;
  // per-pass descriptors are small host tables uploaded per pass
  const char* gk_env = std::getenv("UDA_GKWAY");  // 0: pairwise tree only (A/B and tests)
  const bool gk_on = !(gk_env && *gk_env && std::atoi(gk_env) == 0);
  const bool gk = gk_on && K >= 2 && K <= kGkMaxRuns;
  // chunk = kv_buf - longest record keeps every delivery buffer within kv_buf
  // (the longest record does not depend on the order: max over the side table's record lengths)
  auto chunk_bytes = [&](const Elem*) {
    unsigned int* d_max = reinterpret_cast<unsigned int*>(scan_tmp_.as<int64_t>());
    launch_max_i32(ctx.reclen, total, d_max, s);
    unsigned int m = 0;
    HIP_CHECK(hipMemcpyAsync(&m, d_max, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if ((int64_t)m > kv_buf) throw std::runtime_error("record larger than the delivery buffer");
    return std::max<int64_t>(1, kv_buf - (int64_t)m);
  };
  // F4 for merged elements [e0, e0 + n) whose records start at output byte b0: sizes -> scan ->
  // gather, then the delivery cuts of that range (relative) into host `raw` (pinned; complete once
  // the stream passes this point). Enqueued only.
  auto f4_enqueue = [&](const Elem* order, int64_t e0, int64_t n, int64_t b0, int64_t nbytes, int64_t chunk,
                        int64_t* d_cuts, int64_t* raw) {
    launch_record_sizes(ctx, order + e0, n, sizes_.as<int64_t>() + e0, s);
    launch_exclusive_scan(sizes_.as<int64_t>() + e0, out_off_.as<int64_t>() + e0, n, scan_tmp_.as<int64_t>(), s);
    launch_gather_var(ctx, order + e0, n, out_off_.as<int64_t>() + e0, out + b0, s);
    const int64_t nbuf = (nbytes + chunk - 1) / chunk;
    launch_buffer_cuts(out_off_.as<int64_t>() + e0, n, chunk, nbuf, d_cuts, s);
    HIP_CHECK(hipMemcpyAsync(raw, d_cuts, 8 * (nbuf + 1), hipMemcpyDeviceToHost, s));
    return nbuf;
  };
  auto absolute_cuts = [](const int64_t* raw, int64_t nbuf, int64_t b0, int64_t nbytes, std::vector<int64_t>* cuts) {
    cuts->clear();
    for (int64_t i = 0; i <= nbuf; ++i)
      if (cuts->empty() || b0 + raw[i] != cuts->back()) cuts->push_back(b0 + raw[i]);
    if (cuts->back() != b0 + nbytes) cuts->push_back(b0 + nbytes);
  };
  auto reserve_cuts = [&](int64_t entries) {
    if (cuts_.size() < (size_t)entries * 8) cuts_.alloc((size_t)entries * 8 + 4096);
    if (cuts_host_.size() < (size_t)entries * 8) cuts_host_.alloc((size_t)entries * 8 + 4096);
  };
  int64_t C = 0;
  if (gk && on_round && kway_level(0, cur, eoff, d_eoff, d_eoff, nxt, ctx, s, /*launch_cells=*/false, &C)) {
    // ---- streamed: key-range rounds of cells; round q's output is handed over (on_round) while the
    // device merges round q + 1, so the caller's D2H overlaps the merge
    res.passes = 1;
    const int64_t chunk = chunk_bytes(cur);
    int Q = (int)std::min<int64_t>(C, std::max<int64_t>(1, (bytes + round_bytes - 1) / std::max<int64_t>(round_bytes, 1)));
    std::vector<int64_t> cb(Q + 1);
    for (int q = 0; q <= Q; ++q) cb[q] = C * q / Q;
    if (rounds_.size() < (size_t)(Q + 1) * 24) rounds_.alloc((size_t)(Q + 1) * 24);
    int64_t* d_cb = rounds_.as<int64_t>();
    int64_t* d_re = d_cb + (Q + 1);
    int64_t* d_rb = d_re + (Q + 1);
    HIP_CHECK(hipMemcpyAsync(d_cb, cb.data(), 8 * (Q + 1), hipMemcpyHostToDevice, s));
    launch_gk_round_bounds(gk_[0].split.as<int64_t>(), K, C, d_cb, Q + 1,
                           const_cast<const int64_t* const*>(d_offp), d_re, d_rb, s);
    std::vector<int64_t> re(Q + 1), rb(Q + 1);
    HIP_CHECK(hipMemcpyAsync(re.data(), d_re, 8 * (Q + 1), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(rb.data(), d_rb, 8 * (Q + 1), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemsetAsync(gk_[0].flag.as(), 0, 4, s));
    HIP_CHECK(hipStreamSynchronize(s));
    // per-round slices of the cut buffers, and one completion event per round
    std::vector<int64_t> coff(Q + 1, 0);
    for (int q = 0; q < Q; ++q) coff[q + 1] = coff[q] + (rb[q + 1] - rb[q] + chunk - 1) / chunk + 1;
    reserve_cuts(coff[Q]);
    if ((int)round_ev_.size() < Q)
      for (int q = (int)round_ev_.size(); q < Q; ++q) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        round_ev_.push_back(e);
      }
    std::vector<int64_t> nbufs(Q);
    auto enqueue = [&](int q) {
      launch_gk_cells(ctx, cur, d_eoff, K, gk_[0].split.as<int64_t>(), C, cb[q], cb[q + 1] - cb[q], nxt,
                      gk_[0].flag.as<int>(), s);
      nbufs[q] = f4_enqueue(nxt, re[q], re[q + 1] - re[q], rb[q], rb[q + 1] - rb[q], chunk,
                            cuts_.as<int64_t>() + coff[q], cuts_host_.as<int64_t>() + coff[q]);
      HIP_CHECK(hipEventRecord(round_ev_[(size_t)q], s));
    };
    res.cuts = {0};
    std::vector<int64_t> rc;
    enqueue(0);
    for (int q = 0; q < Q; ++q) {
      if (q + 1 < Q) enqueue(q + 1);  // the device runs ahead while round q is delivered
      HIP_CHECK(hipEventSynchronize(round_ev_[(size_t)q]));
      int overflow = 0;
      HIP_CHECK(hipMemcpy(&overflow, gk_[0].flag.as(), 4, hipMemcpyDeviceToHost));
      if (overflow) throw std::runtime_error("generic k-way: a cell above capacity in a streamed round");
      absolute_cuts(cuts_host_.as<int64_t>() + coff[q], nbufs[q], rb[q], rb[q + 1] - rb[q], &rc);
      on_round(rc, re[q + 1] - re[q], q + 1 == Q);
      res.cuts.insert(res.cuts.end(), rc.begin() + 1, rc.end());
    }
    HIP_CHECK(hipStreamSynchronize(s));
    phase("f3_f4_rounds");
  } else {
    // ---- whole: F3 (K-way, else the pairwise tree), then F4 over everything
    bool merged = false;
    if (gk) {
      if (kway_level(0, cur, eoff, d_eoff, d_eoff, nxt, ctx, s, /*launch_cells=*/true, &C)) {
        std::swap(cur, nxt);
        res.passes = 1;
        merged = true;
      } else {
        UDA_LOG(kWarn, "generic k-way: a cell above capacity, falling back to the pairwise merge");
      }
    }
    for (const PassDesc& pd : merged ? std::vector<PassDesc>{}
                                     : upload_passes(plan_merge_passes(eoff, {0, (int)eoff.size() - 1}, kGenericMergeTile),
                                                     passtab_, s)) {
      launch_merge_partition_generic(cur, pd, splits_.as<int64_t>(), ctx, s);
      launch_merge_pass_generic(cur, nxt, pd, splits_.as<int64_t>(), ctx, s);
      std::swap(cur, nxt);
      ++res.passes;
    }
    phase("f3_merge");
    const int64_t chunk = chunk_bytes(cur);
    const int64_t nbuf = (bytes + chunk - 1) / chunk;
    reserve_cuts(nbuf + 1);
    f4_enqueue(cur, 0, total, 0, bytes, chunk, cuts_.as<int64_t>(), cuts_host_.as<int64_t>());
    HIP_CHECK(hipStreamSynchronize(s));
    absolute_cuts(cuts_host_.as<int64_t>(), nbuf, 0, bytes, &res.cuts);
    if (on_round) on_round(res.cuts, total, true);
  }
  phase("f4_gather_cuts");
  if (prof) {
    std::string line = "[GM profile] runs=" + std::to_string(K) + " records=" + std::to_string(total) +
                       " serial_runs=" + std::to_string(f1_serial_runs_);
    for (auto& ph : phases) line += " " + std::string(ph.first) + "=" + std::to_string(ph.second).substr(0, 6) + "ms";
    fprintf(stderr, "%s\n", line.c_str());
  }
  return res;
}

}  // namespace gpu
}  // namespace uda
