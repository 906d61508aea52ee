#include "generic_merger.h"

#include <algorithm>
#include <stdexcept>

namespace uda {
namespace gpu {

void GenericMerger::reserve(int64_t records, int runs) {
  if (records <= cap_records_ && runs <= cap_runs_) return;
  records = std::max<int64_t>(records, 1);
  const int64_t max_tiles = records / kMergeTile + runs + 2;
  elems_a_.alloc((size_t)records * sizeof(Elem));
  elems_b_.alloc((size_t)records * sizeof(Elem));
  splits_.alloc((size_t)max_tiles * 8);
  sizes_.alloc((size_t)records * 8);
  out_off_.alloc((size_t)(std::max<int64_t>(records, runs) + 1) * 8);  // also holds elem_off (runs+1)
  scan_tmp_.alloc((size_t)scan_tmp_elems(records) * 8);
  cap_records_ = records;
  cap_runs_ = std::max(runs, cap_runs_);
}

GenericMergeResult GenericMerger::merge(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                                        int kind, uint8_t* out, int64_t out_cap, int64_t kv_buf, hipStream_t s) {
  GenericMergeResult res;
  const int K = (int)runs.size();
  if (K == 0) {
    res.cuts = {0};
    return res;
  }
  if (K > 65536) throw std::runtime_error("GenericMerger: at most 65536 runs");
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
  // ---- F1 pass 1: count
  launch_count_records(d_bases, d_nbytes, K, d_counts, d_recb, d_status, s);
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
    if (counts[k] > 0xFFFFFFFFll) throw std::runtime_error("GenericMerger: run has more than 2^32 records");
    eoff[k + 1] = eoff[k] + counts[k];
    bytes += recb[k];
  }
  const int64_t total = eoff[K];
  if (bytes > out_cap) throw std::runtime_error("GenericMerger: output capacity too small");
  res.records = total;
  res.bytes = bytes;
  reserve(total, K);
  // offsets storage: run k gets counts[k]+1 entries
  const int64_t off_elems = total + K;
  if (offsets_.size() < (size_t)off_elems * 8) offsets_.alloc((size_t)off_elems * 8);
  std::vector<int64_t*> offp(K);
  for (int k = 0; k < K; ++k) offp[k] = offsets_.as<int64_t>() + eoff[k] + k;
  HIP_CHECK(hipMemcpyAsync(d_offp, offp.data(), 8 * K, hipMemcpyHostToDevice, s));
  // ---- F1 pass 2: offsets
  launch_index_records(d_bases, d_nbytes, K, d_offp, s);
  GenericKeyCtx ctx{d_bases, const_cast<const int64_t* const*>(d_offp), kind};
  if (total == 0) {
    res.cuts = {0};
    return res;
  }
  // ---- F2: normalize (elem_off goes into the out_off scratch, reused below)
  int64_t* d_eoff = out_off_.as<int64_t>();
  HIP_CHECK(hipMemcpyAsync(d_eoff, eoff.data(), 8 * (K + 1), hipMemcpyHostToDevice, s));
  Elem* cur = elems_a_.as<Elem>();
  Elem* nxt = elems_b_.as<Elem>();
  launch_normalize_generic(ctx, d_eoff, K, total, cur, s);
  // ---- F3: merge tree; per-pass descriptors are small host tables uploaded per pass
  std::vector<int64_t> seg(eoff);
  std::vector<DeviceBuffer> pass_tabs;
  while ((int)seg.size() - 1 > 1) {
    const int S = (int)seg.size() - 1;
    const int P = (S + 1) / 2;
    std::vector<int64_t> tab(S + 1 + P + 1);
    std::copy(seg.begin(), seg.end(), tab.begin());
    int64_t* tp = tab.data() + S + 1;
    tp[0] = 0;
    std::vector<int64_t> next{0};
    for (int p = 0; p < P; ++p) {
      const int64_t beg = seg[2 * p], end = seg[std::min(2 * p + 2, S)];
      tp[p + 1] = tp[p] + (end - beg + kMergeTile - 1) / kMergeTile;
      next.push_back(end);
    }
    pass_tabs.emplace_back(tab.size() * 8);
    HIP_CHECK(hipMemcpyAsync(pass_tabs.back().as(), tab.data(), tab.size() * 8, hipMemcpyHostToDevice, s));
    PassDesc pd;
    pd.seg_off = pass_tabs.back().as<int64_t>();
    pd.tile_prefix = pass_tabs.back().as<int64_t>() + S + 1;
    pd.nseg = S;
    pd.npairs = P;
    pd.ntiles = (int)tp[P];
    launch_merge_partition_generic(cur, pd, splits_.as<int64_t>(), ctx, s);
    launch_merge_pass_generic(cur, nxt, pd, splits_.as<int64_t>(), ctx, s);
    std::swap(cur, nxt);
    seg.swap(next);
    ++res.passes;
  }
  // ---- F4: sizes in merged order -> scan -> gather
  launch_record_sizes(ctx, cur, total, sizes_.as<int64_t>(), s);
  launch_exclusive_scan(sizes_.as<int64_t>(), out_off_.as<int64_t>(), total, scan_tmp_.as<int64_t>(), s);
  launch_gather_var(ctx, cur, total, out_off_.as<int64_t>(), out, s);
  // ---- delivery cuts: records whose output offset starts in [j*chunk, (j+1)*chunk) form buffer j;
  // chunk = kv_buf - longest record keeps every buffer within kv_buf
  int64_t max_rec = 0;
  {
    unsigned long long* d_max = reinterpret_cast<unsigned long long*>(scan_tmp_.as<int64_t>());  // free again
    launch_max_i64(sizes_.as<int64_t>(), total, d_max, s);
    unsigned long long m = 0;
    HIP_CHECK(hipMemcpyAsync(&m, d_max, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    max_rec = (int64_t)m;
  }
  if (max_rec > kv_buf) throw std::runtime_error("record larger than the delivery buffer");
  const int64_t chunk = std::max<int64_t>(1, kv_buf - max_rec);
  const int64_t nbuf = (bytes + chunk - 1) / chunk;
  if (cuts_.size() < (size_t)(nbuf + 1) * 8) cuts_.alloc((size_t)(nbuf + 1) * 8);
  launch_buffer_cuts(out_off_.as<int64_t>(), total, chunk, nbuf, cuts_.as<int64_t>(), s);
  std::vector<int64_t> raw(nbuf + 1);
  HIP_CHECK(hipMemcpyAsync(raw.data(), cuts_.as(), 8 * (nbuf + 1), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  res.cuts.clear();
  for (int64_t b : raw)
    if (res.cuts.empty() || b != res.cuts.back()) res.cuts.push_back(b);
  if (res.cuts.back() != bytes) res.cuts.push_back(bytes);
  return res;
}

}  // namespace gpu
}  // namespace uda
