// Device k-way merge of arbitrary IFile runs (any supported key class, variable-length records).
// Used by the NetMerger's GPU backend (mapred.uda.merge.backend=gpu) and the secondary-sort config.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

#include "device_engine.h"
#include "kernels.h"

namespace uda {
namespace gpu {

struct GenericMergeResult {
  int64_t records = 0;
  int64_t bytes = 0;     // merged record bytes (no EOF marker)
  int passes = 0;
  std::vector<int64_t> cuts;  // delivery buffer boundaries as byte offsets into the output (0 .. bytes)
};

class GenericMerger {
 public:
  GenericMerger() = default;
  ~GenericMerger();
  GenericMerger(const GenericMerger&) = delete;
  GenericMerger& operator=(const GenericMerger&) = delete;
  // runs: device pointers to IFile streams (records, optionally followed by the EOF marker).
  // Merged records are written to `out` (capacity out_cap). Buffer cuts are chosen so that every
  // delivery buffer holds whole records and at most `kv_buf` bytes (EOF added by the caller).
  // Synchronizes `s` (the record counts size the workspace).
  //
  // on_round (optional): the output is handed over in key-range rounds of about round_bytes as they
  // complete: on_round(cuts, records, last) with absolute cuts of that round's delivery buffers, called
  // on this thread while the device already merges the next round (so a caller's D2H of the round
  // overlaps the merge). Without the single-pass path it is called once for the whole output.
  using RoundFn = std::function<void(const std::vector<int64_t>& cuts, int64_t records, bool last)>;
  GenericMergeResult merge(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                           int kind, uint8_t* out, int64_t out_cap, int64_t kv_buf, hipStream_t s,
                           const RoundFn& on_round = nullptr, int64_t round_bytes = 256ll << 20);

  // runs the last merge indexed with the serial F1 walk (records longer than the parallel entry table)
  int f1_serial_runs() const { return f1_serial_runs_; }
  // device bytes held by this merger's workspaces
  int64_t workspace_bytes() const;

 private:
  int f1_serial_runs_ = 0;
  void reserve(int64_t records, int runs);
  DeviceBuffer eoff_, rounds_, passtab_;  // passtab_: pairwise-tree pass tables (no hipMalloc/hipFree per merge)
  PinnedBuffer cuts_host_;
  std::vector<hipEvent_t> round_ev_;
  DeviceBuffer elems_a_, elems_b_, splits_, sizes_, out_off_, scan_tmp_, cuts_, offsets_, tables_, side_, ck_, f1ws_;
  // single-pass K-way (generic_kway.hip), per recursion level: sample offsets, per-run samples,
  // merged samples (ping-pong), splitters, per-run cell splits, sample histogram, overflow flag
  struct KwayBuffers {
    DeviceBuffer tab, samp, sa, sb, bounds, split, hist, flag, passtab;
  };
  std::vector<KwayBuffers> gk_;
  static constexpr int64_t kGkRecurseSamples = 1 << 18;  // larger samples are merged by a K-way level
  // d_off: element offsets of the level's runs; d_ord_off: run boundaries in record ordinals (level 0)
  // launch_cells false: stop after the level's splits (gk_[0].split, *cells cells) for a streamed merge.
  bool kway_level(int depth, const Elem* in, const std::vector<int64_t>& off, const int64_t* d_off,
                  const int64_t* d_ord_off, Elem* out, const GenericKeyCtx& ctx, hipStream_t s,
                  bool launch_cells = true, int64_t* cells = nullptr);
  int64_t cap_records_ = 0;
  int cap_runs_ = 0;
};

}  // namespace gpu
}  // namespace uda
