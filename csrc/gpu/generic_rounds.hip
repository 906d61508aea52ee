// Key-range round planning for the generic device merge. See generic_rounds.h.
#include "generic_rounds.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>

#include "kernels.h"
#include "uda/compare.h"
#include "uda/log.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {
constexpr int kSampleKey = 64;      // content bytes kept per sampled key (a bound may be any byte string)
constexpr int kSamplesPerRound = 512;

// Key content of the record at p (n bytes of stream left): pointer and length.
__device__ __forceinline__ const uint8_t* rec_key(const uint8_t* p, int64_t n, int kind, int* len, int64_t* size) {
  int64_t kl = 0, vl = 0;
  const int a = vint_decode(p, (size_t)(n < 9 ? n : 9), &kl);
  const int b = vint_decode(p + a, (size_t)(n - a < 9 ? n - a : 9), &vl);
  const uint8_t* key = p + a + b;
  const int o = key_content_offset((KeyKind)kind, key, (int)kl);
  *len = (int)kl - o;
  *size = a + b + kl + vl;
  return key + o;
}

// sign of key - bound in the key order (content bytes, then length)
__device__ __forceinline__ int cmp_bound(const uint8_t* k, int kl, const uint8_t* b, int bl) {
  const int n = kl < bl ? kl : bl;
  for (int i = 0; i < n; ++i)
    if (k[i] != b[i]) return (int)k[i] - (int)b[i];
  return kl - bl;
}

// first chunk >= c of the run (chunks [c, end)) in which a record starts; end if none
__device__ __forceinline__ int64_t next_rec_chunk(const int64_t* ck_count, int64_t c, int64_t end) {
  while (c < end && ck_count[c] == 0) ++c;
  return c;
}

__global__ void __launch_bounds__(256) gr_sample_kernel(uint8_t* const* bases, const int64_t* rec_bytes,
                                                        const int64_t* chunk_base, const int64_t* ck_start,
                                                        const int64_t* ck_count, const int64_t* samp_chunk,
                                                        const int32_t* samp_run, int ns, int kind, uint8_t* keys,
                                                        int32_t* klen) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ns) return;
  const int r = samp_run[i];
  const int64_t c = next_rec_chunk(ck_count, samp_chunk[i], chunk_base[r + 1]);
  klen[i] = -1;
  if (c >= chunk_base[r + 1]) return;
  const int64_t pos = ck_start[c];
  if (pos >= rec_bytes[r]) return;  // the EOF marker
  int len = 0;
  int64_t size = 0;
  const uint8_t* k = rec_key(bases[r] + pos, rec_bytes[r] - pos, kind, &len, &size);
  const int n = len < kSampleKey ? len : kSampleKey;
  for (int j = 0; j < n; ++j) keys[(int64_t)i * kSampleKey + j] = k[j];
  klen[i] = n;
}

// out[r * (nb + 2) + 1 + b]: byte offset of the first record of run r whose key is not below bound b
__global__ void __launch_bounds__(64) gr_split_kernel(uint8_t* const* bases, const int64_t* rec_bytes,
                                                      const int64_t* chunk_base, const int64_t* ck_start,
                                                      const int64_t* ck_count, int nruns, int kind,
                                                      const uint8_t* bound_bytes, const int32_t* bound_off, int nb,
                                                      int64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nruns * nb) return;
  const int r = (int)(t / nb), bi = (int)(t % nb);
  const uint8_t* bnd = bound_bytes + bound_off[bi];
  const int bl = bound_off[bi + 1] - bound_off[bi];
  const uint8_t* p = bases[r];
  const int64_t rb = rec_bytes[r];
  const int64_t lo = chunk_base[r], hi = chunk_base[r + 1];
  // not-below(c): the first record starting at or after chunk c has a key >= bound (true past the end)
  auto not_below = [&](int64_t c) {
    const int64_t cc = next_rec_chunk(ck_count, c, hi);
    if (cc >= hi) return true;
    const int64_t pos = ck_start[cc];
    if (pos >= rb) return true;
    int len = 0;
    int64_t size = 0;
    const uint8_t* k = rec_key(p + pos, rb - pos, kind, &len, &size);
    return cmp_bound(k, len, bnd, bl) >= 0;
  };
  int64_t a = lo, b = hi;  // smallest c in [lo, hi] with not_below(c) (not_below(hi) is true)
  while (a < b) {
    const int64_t m = a + ((b - a) >> 1);
    if (not_below(m))
      b = m;
    else
      a = m + 1;
  }
  int64_t pos = 0, end = rb;
  if (a < hi) {
    const int64_t cc = next_rec_chunk(ck_count, a, hi);
    end = cc < hi ? ck_start[cc] : rb;
    if (end > rb) end = rb;
  }
  if (a > lo) {  // chunk a-1's first record is below the bound: start there (a record starts in it or before)
    int64_t c = a - 1;
    while (c > lo && ck_count[c] == 0) --c;
    pos = ck_count[c] > 0 ? ck_start[c] : 0;
    while (pos < end) {
      int len = 0;
      int64_t size = 0;
      const uint8_t* k = rec_key(p + pos, rb - pos, kind, &len, &size);
      if (cmp_bound(k, len, bnd, bl) >= 0) break;
      pos += size;
    }
  }
  out[(int64_t)r * (nb + 2) + 1 + bi] = pos < end ? pos : end;
}

// Key of the last complete record of each run (up to kSampleKey content bytes; klen -1 if the run has
// none): the last chunk in which a record starts below rec_bytes, then a walk to the last start.
__global__ void __launch_bounds__(64) gr_lastkey_kernel(uint8_t* const* bases, const int64_t* rec_bytes,
                                                        const int64_t* chunk_base, const int64_t* ck_start,
                                                        const int64_t* ck_count, int nruns, int kind,
                                                        int64_t chunk_bytes, uint8_t* keys, int32_t* klen) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  klen[r] = -1;
  const int64_t rb = rec_bytes[r];
  if (rb <= 0) return;
  const int64_t lo = chunk_base[r];
  int64_t c = lo + (rb - 1) / chunk_bytes;
  if (c >= chunk_base[r + 1]) c = chunk_base[r + 1] - 1;
  while (c >= lo && (ck_count[c] == 0 || ck_start[c] >= rb)) --c;
  if (c < lo) return;
  const uint8_t* p = bases[r];
  int64_t pos = ck_start[c], last = pos;
  while (pos < rb) {
    int len = 0;
    int64_t size = 0;
    (void)rec_key(p + pos, rb - pos, kind, &len, &size);
    if (size <= 0) break;
    last = pos;
    pos += size;
  }
  int len = 0;
  int64_t size = 0;
  const uint8_t* k = rec_key(p + last, rb - last, kind, &len, &size);
  const int n = len < kSampleKey ? len : kSampleKey;
  for (int j = 0; j < n; ++j) keys[(int64_t)r * kSampleKey + j] = k[j];
  klen[r] = n;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void ensure(DeviceBuffer& b, size_t bytes) {
  if (b.size() < bytes) b.alloc(bytes + bytes / 8 + 256);
}
struct F1Dev {
  int64_t nchunks = 0;
  std::vector<int64_t> chunk_base;
  std::vector<int32_t> chunk_run;
  uint8_t** d_bases = nullptr;
  int64_t *d_nbytes = nullptr, *d_counts = nullptr, *d_recb = nullptr, *d_cbase = nullptr;
  int64_t *d_ckstart = nullptr, *d_ckcount = nullptr;
  int* d_status = nullptr;
};

// F1 pass 1 over the runs (chunk checkpoints, record bytes per run) in the planner's workspace.
// partial: runs are landed prefixes (a record cut by the end is not counted). Synchronizes `s`;
// throws on a corrupt run.
F1Dev f1_checkpoints(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes, int kind,
                     bool partial, GenericRoundsWs& ws, hipStream_t s) {
  F1Dev f;
  const int K = (int)runs.size();
  const int64_t CH = f1_chunk_bytes();
  std::vector<int64_t>& chunk_base = f.chunk_base;
  chunk_base.assign(K + 1, 0);
  for (int k = 0; k < K; ++k) chunk_base[k + 1] = chunk_base[k] + (run_bytes[k] + CH - 1) / CH;
  const int64_t nchunks = chunk_base[K];
  f.nchunks = nchunks;
  if (nchunks == 0) return f;
  std::vector<int32_t>& chunk_run = f.chunk_run;
  chunk_run.resize((size_t)nchunks);
  for (int k = 0; k < K; ++k)
    for (int64_t c = chunk_base[k]; c < chunk_base[k + 1]; ++c) chunk_run[(size_t)c] = k;
  const int64_t SC = f1_super_chunks();
  std::vector<int64_t> sup_base(K + 1, 0);
  for (int k = 0; k < K; ++k) sup_base[k + 1] = sup_base[k] + (chunk_base[k + 1] - chunk_base[k] + SC - 1) / SC;
  const int64_t nsup = sup_base[K];
  std::vector<int32_t> sup_run((size_t)std::max<int64_t>(nsup, 1));
  for (int k = 0; k < K; ++k)
    for (int64_t j = sup_base[k]; j < sup_base[k + 1]; ++j) sup_run[(size_t)j] = k;

  ensure(ws.tables, (size_t)K * 8 * 6 + 256);
  uint8_t* t = ws.tables.as<uint8_t>();
  auto* d_bases = reinterpret_cast<uint8_t**>(t);
  auto* d_nbytes = reinterpret_cast<int64_t*>(t + 8 * (size_t)K);
  auto* d_counts = reinterpret_cast<int64_t*>(t + 16 * (size_t)K);
  auto* d_recb = reinterpret_cast<int64_t*>(t + 24 * (size_t)K);
  auto* d_status = reinterpret_cast<int*>(t + 32 * (size_t)K);
  auto* d_cbase = reinterpret_cast<int64_t*>(t + 40 * (size_t)K + 64);  // K + 1
  ensure(ws.ck, (size_t)nchunks * (8 + 8 + 4) + 256);
  int64_t* d_ckstart = ws.ck.as<int64_t>();
  int64_t* d_ckcount = d_ckstart + nchunks;
  int32_t* d_crun = reinterpret_cast<int32_t*>(d_ckcount + nchunks);
  HIP_CHECK(hipMemcpyAsync(d_bases, runs.data(), 8 * (size_t)K, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_nbytes, run_bytes.data(), 8 * (size_t)K, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_cbase, chunk_base.data(), 8 * (size_t)(K + 1), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_crun, chunk_run.data(), 4 * (size_t)nchunks, hipMemcpyHostToDevice, s));
  const size_t wsb = f1_parallel_workspace(nchunks, nsup) + (size_t)(K + 1) * 8 + (size_t)(nsup + 1) * 4 + 512;
  ensure(ws.f1ws, wsb);
  uint8_t* w = ws.f1ws.as<uint8_t>();
  auto* d_supbase = reinterpret_cast<int64_t*>(w);
  auto* d_suprun = reinterpret_cast<int32_t*>(w + (size_t)(K + 1) * 8);
  uint8_t* d_fws = w + (((size_t)(K + 1) * 8 + (size_t)(nsup + 1) * 4 + 255) & ~(size_t)255);
  HIP_CHECK(hipMemcpyAsync(d_supbase, sup_base.data(), 8 * (size_t)(K + 1), hipMemcpyHostToDevice, s));
  if (nsup > 0) HIP_CHECK(hipMemcpyAsync(d_suprun, sup_run.data(), 4 * (size_t)nsup, hipMemcpyHostToDevice, s));
  launch_f1_parallel(d_bases, d_nbytes, K, d_cbase, d_crun, nchunks, d_supbase, d_suprun, nsup, d_fws, d_ckstart,
                     d_ckcount, d_counts, d_recb, d_status, s, kind, partial);
  std::vector<int> status(K);
  HIP_CHECK(hipMemcpyAsync(status.data(), d_status, 4 * (size_t)K, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<int> redo;
  for (int k = 0; k < K; ++k)
    if (status[k] == 2) redo.push_back(k);
  if (!redo.empty()) {  // records longer than the chunk-function table: the serial walk
    DeviceBuffer d_redo(redo.size() * 4);
    HIP_CHECK(hipMemcpyAsync(d_redo.as(), redo.data(), redo.size() * 4, hipMemcpyHostToDevice, s));
    launch_f1_scan(d_bases, d_nbytes, (int)redo.size(), d_cbase, d_ckstart, d_ckcount, d_counts, d_recb, d_status, s,
                   nullptr, d_redo.as<int>(), partial);
    HIP_CHECK(hipMemcpyAsync(status.data(), d_status, 4 * (size_t)K, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  for (int k = 0; k < K; ++k)
    if (status[k] != 0) throw std::runtime_error("round planning: corrupt or truncated IFile run " + std::to_string(k));
  f.d_bases = d_bases;
  f.d_nbytes = d_nbytes;
  f.d_counts = d_counts;
  f.d_recb = d_recb;
  f.d_status = d_status;
  f.d_cbase = d_cbase;
  f.d_ckstart = d_ckstart;
  f.d_ckcount = d_ckcount;
  return f;
}
}  // namespace

GenericRoundsPlan plan_generic_rounds(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                                      int kind, int64_t round_bytes, GenericRoundsWs& ws, hipStream_t s) {
  const double t0 = now_ms();
  GenericRoundsPlan plan;
  const int K = (int)runs.size();
  int64_t total = 0;
  for (int64_t b : run_bytes) total += b;
  const int want = (int)std::max<int64_t>(1, (total + std::max<int64_t>(round_bytes, 1) - 1) / std::max<int64_t>(round_bytes, 1));
  auto trivial = [&] {
    plan.rounds = 1;
    plan.pos.assign((size_t)K * 2, 0);
    for (int k = 0; k < K; ++k) plan.pos[(size_t)k * 2 + 1] = run_bytes[k];
    plan.max_round_bytes = total;
    plan.plan_ms = now_ms() - t0;
    return plan;
  };
  if (want <= 1 || K == 0) return trivial();

  // ---- F1 checkpoints of the whole runs (pass 1 only)
  F1Dev f = f1_checkpoints(runs, run_bytes, kind, false, ws, s);
  const int64_t nchunks = f.nchunks;
  if (nchunks == 0) return trivial();
  const std::vector<int32_t>& chunk_run = f.chunk_run;
  uint8_t** d_bases = f.d_bases;
  int64_t *d_recb = f.d_recb, *d_cbase = f.d_cbase, *d_ckstart = f.d_ckstart, *d_ckcount = f.d_ckcount;

  // ---- sample chunk-leading keys (chunks spread evenly over all input bytes)
  const int64_t ns = std::min<int64_t>(nchunks, (int64_t)want * kSamplesPerRound);
  std::vector<int64_t> samp_chunk((size_t)ns);
  std::vector<int32_t> samp_run((size_t)ns);
  for (int64_t i = 0; i < ns; ++i) {
    const int64_t c = (2 * i + 1) * nchunks / (2 * ns);
    samp_chunk[(size_t)i] = c;
    samp_run[(size_t)i] = chunk_run[(size_t)c];
  }
  ensure(ws.samp, (size_t)ns * (8 + 4 + 4 + kSampleKey) + 256);
  auto* d_sc = ws.samp.as<int64_t>();
  auto* d_sr = reinterpret_cast<int32_t*>(d_sc + ns);
  auto* d_kl = d_sr + ns;
  auto* d_keys = reinterpret_cast<uint8_t*>(d_kl + ns);
  HIP_CHECK(hipMemcpyAsync(d_sc, samp_chunk.data(), 8 * (size_t)ns, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_sr, samp_run.data(), 4 * (size_t)ns, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(gr_sample_kernel, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, d_bases, d_recb, d_cbase,
                     d_ckstart, d_ckcount, d_sc, d_sr, (int)ns, kind, d_keys, d_kl);
  HIP_CHECK(hipGetLastError());
  std::vector<int32_t> kl((size_t)ns);
  std::vector<uint8_t> keys((size_t)ns * kSampleKey);
  HIP_CHECK(hipMemcpyAsync(kl.data(), d_kl, 4 * (size_t)ns, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(keys.data(), d_keys, keys.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<std::string> sk;
  sk.reserve((size_t)ns);
  for (int64_t i = 0; i < ns; ++i)
    if (kl[(size_t)i] >= 0) sk.emplace_back(reinterpret_cast<const char*>(&keys[(size_t)i * kSampleKey]), (size_t)kl[(size_t)i]);
  std::sort(sk.begin(), sk.end());  // unsigned bytewise, a prefix first: the key order on content
  // round 0 takes an eighth of a round's share: its merge is the only one not overlapped with a
  // delivery, so the consumer starts early; rounds 1..want split the rest evenly
  std::vector<std::string> bounds;
  std::vector<double> cut;
  const double first = 1.0 / (8.0 * want);
  cut.push_back(first);
  for (int q = 1; q < want; ++q) cut.push_back(first + (1.0 - first) * q / want);
  for (double f : cut) {
    if (sk.empty()) break;
    const std::string& b = sk[(size_t)std::min<int64_t>((int64_t)sk.size() - 1, (int64_t)(f * (double)sk.size()))];
    if (bounds.empty() || b > bounds.back()) bounds.push_back(b);
  }
  if (bounds.empty()) return trivial();
  const int nb = (int)bounds.size();
  std::vector<int32_t> boff(nb + 1, 0);
  std::string packed;
  for (int b = 0; b < nb; ++b) {
    packed += bounds[(size_t)b];
    boff[b + 1] = (int32_t)packed.size();
  }
  ensure(ws.bounds, packed.size() + 4 * (size_t)(nb + 1) + 64);
  auto* d_boff = ws.bounds.as<int32_t>();
  auto* d_bb = reinterpret_cast<uint8_t*>(d_boff + nb + 1);
  HIP_CHECK(hipMemcpyAsync(d_boff, boff.data(), 4 * (size_t)(nb + 1), hipMemcpyHostToDevice, s));
  if (!packed.empty()) HIP_CHECK(hipMemcpyAsync(d_bb, packed.data(), packed.size(), hipMemcpyHostToDevice, s));
  ensure(ws.out, 8 * (size_t)K * (nb + 2));
  const int64_t nt = (int64_t)K * nb;
  hipLaunchKernelGGL(gr_split_kernel, dim3((unsigned)((nt + 63) / 64)), dim3(64), 0, s, d_bases, d_recb, d_cbase,
                     d_ckstart, d_ckcount, K, kind, d_bb, d_boff, nb, ws.out.as<int64_t>());
  HIP_CHECK(hipGetLastError());
  plan.rounds = nb + 1;
  plan.pos.assign((size_t)K * (nb + 2), 0);
  HIP_CHECK(hipMemcpyAsync(plan.pos.data(), ws.out.as(), 8 * plan.pos.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  for (int k = 0; k < K; ++k) {
    plan.pos[(size_t)k * (nb + 2)] = 0;
    plan.pos[(size_t)k * (nb + 2) + nb + 1] = run_bytes[k];
    for (int q = 0; q <= nb; ++q)
      if (plan.pos[(size_t)k * (nb + 2) + q + 1] < plan.pos[(size_t)k * (nb + 2) + q])
        throw std::runtime_error("round planning: split positions out of order in run " + std::to_string(k));
  }
  for (int q = 0; q < plan.rounds; ++q) {
    int64_t b = 0;
    for (int k = 0; k < K; ++k) b += plan.at(k, q + 1) - plan.at(k, q);
    plan.max_round_bytes = std::max(plan.max_round_bytes, b);
  }
  plan.plan_ms = now_ms() - t0;
  return plan;
}

ProgressiveSplit plan_progressive_split(const std::vector<const uint8_t*>& windows, const std::vector<int64_t>& avail,
                                        const std::vector<char>& final_run, int kind, GenericRoundsWs& ws,
                                        hipStream_t s) {
  const double t0 = now_ms();
  ProgressiveSplit ps;
  const int K = (int)windows.size();
  ps.complete.assign(K, 0);
  ps.split.assign(K, 0);
  F1Dev f = f1_checkpoints(windows, avail, kind, true, ws, s);
  if (f.nchunks == 0) {
    ps.ms = now_ms() - t0;
    return ps;
  }
  HIP_CHECK(hipMemcpyAsync(ps.complete.data(), f.d_recb, 8 * (size_t)K, hipMemcpyDeviceToHost, s));
  ensure(ws.samp, (size_t)K * (4 + kSampleKey) + 256);
  auto* d_kl = ws.samp.as<int32_t>();
  auto* d_keys = reinterpret_cast<uint8_t*>(d_kl + K + 16);
  hipLaunchKernelGGL(gr_lastkey_kernel, dim3((unsigned)((K + 63) / 64)), dim3(64), 0, s, f.d_bases, f.d_recb, f.d_cbase,
                     f.d_ckstart, f.d_ckcount, K, kind, f1_chunk_bytes(), d_keys, d_kl);
  HIP_CHECK(hipGetLastError());
  std::vector<int32_t> kl((size_t)K);
  std::vector<uint8_t> keys((size_t)K * kSampleKey);
  HIP_CHECK(hipMemcpyAsync(kl.data(), d_kl, 4 * (size_t)K, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(keys.data(), d_keys, keys.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  // bound: the least last-complete key over the windows that do not reach their run's end; every
  // record below it has landed (a run's later records are >= its last landed key >= the bound)
  bool have = false, all_final = true;
  std::string bound;
  for (int k = 0; k < K; ++k) {
    if (final_run[(size_t)k]) continue;
    all_final = false;
    if (kl[(size_t)k] < 0) {  // nothing complete landed yet in this window: no record is safe to merge
      ps.ms = now_ms() - t0;
      return ps;
    }
    std::string key(reinterpret_cast<const char*>(&keys[(size_t)k * kSampleKey]), (size_t)kl[(size_t)k]);
    if (!have || key < bound) bound = std::move(key);
    have = true;
  }
  if (all_final) {  // the rest of every run: no bound
    ps.split = ps.complete;
    ps.bounded = false;
    ps.ms = now_ms() - t0;
    return ps;
  }
  ps.bounded = true;
  ps.bound = bound;
  const int32_t boff[2] = {0, (int32_t)bound.size()};
  ensure(ws.bounds, bound.size() + 8 + 64);
  auto* d_boff = ws.bounds.as<int32_t>();
  auto* d_bb = reinterpret_cast<uint8_t*>(d_boff + 2);
  HIP_CHECK(hipMemcpyAsync(d_boff, boff, 8, hipMemcpyHostToDevice, s));
  if (!bound.empty()) HIP_CHECK(hipMemcpyAsync(d_bb, bound.data(), bound.size(), hipMemcpyHostToDevice, s));
  ensure(ws.out, 8 * (size_t)K * 3);
  hipLaunchKernelGGL(gr_split_kernel, dim3((unsigned)((K + 63) / 64)), dim3(64), 0, s, f.d_bases, f.d_recb, f.d_cbase,
                     f.d_ckstart, f.d_ckcount, K, kind, d_bb, d_boff, 1, ws.out.as<int64_t>());
  HIP_CHECK(hipGetLastError());
  std::vector<int64_t> pos((size_t)K * 3);
  HIP_CHECK(hipMemcpyAsync(pos.data(), ws.out.as(), 8 * pos.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  for (int k = 0; k < K; ++k) {
    const int64_t v = pos[(size_t)k * 3 + 1];
    if (v < 0 || v > ps.complete[(size_t)k]) throw std::runtime_error("progressive split out of range in run " + std::to_string(k));
    ps.split[(size_t)k] = v;
  }
  ps.ms = now_ms() - t0;
  return ps;
}

}  // namespace gpu
}  // namespace uda
