// Key-range rounds for the generic (any key class, variable-length records) device merge: the
// working set of a reduce task is bounded by `round_bytes`, not by its partition size.
//
// Reference: the reducer's memory-bounded merge (buffer sizing in handle_init_msg,
// src/Merger/reducer.cc:102-120, and the hybrid LPQ/RPQ of MergeManager.cc:202-288) with the key
// comparator of CompareFunc.cc:70-91. Here the partitions stay where they are (HBM of the provider,
// or the staged copy) and the merge walks them in Q key ranges:
//   1. F1 checkpoints of every run (first record start and record count per 4 KiB chunk, the same
//      parallel chunk-function composition the merge uses) - 28 bytes per 4 KiB of input;
//   2. a regular sample of chunk-leading keys (up to kSampleKey content bytes each), sorted on the
//      host with the key order, gives Q-1 bound strings of about equal input bytes per round;
//   3. one lane per (run, bound) finds the byte position of the first record whose key is not below
//      the bound: a binary search over the chunk checkpoints, then a walk of at most one chunk.
// Round q merges the byte slices [pos(k, q), pos(k, q+1)) of every run k. Every run is split by the
// same bound strings under the same order, so the concatenated rounds are the total order. A bound is
// any byte string (a truncated sample is fine); equal keys never straddle a bound.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "device_engine.h"

namespace uda {
namespace gpu {

struct GenericRoundsPlan {
  int rounds = 1;
  std::vector<int64_t> pos;  // [run][round 0..Q]: byte offsets (pos(k, Q) = run bytes)
  int64_t max_round_bytes = 0;
  double plan_ms = 0;
  int64_t at(int k, int q) const { return pos[(size_t)k * (rounds + 1) + q]; }
};

// Scratch of the planner (reused across tasks).
struct GenericRoundsWs {
  DeviceBuffer tables, ck, f1ws, samp, bounds, out;
};

// Plan Q = ceil(total / round_bytes) rounds (fewer if the keys do not allow more distinct bounds).
// runs: device pointers to IFile streams (records, optionally followed by the EOF marker).
// Synchronizes `s`.
GenericRoundsPlan plan_generic_rounds(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                                      int kind, int64_t round_bytes, GenericRoundsWs& ws, hipStream_t s);

// Progressive merging of runs that are still arriving (a reduce task whose partitions land over PCIe
// while the merged output goes back the other way). windows[k]: device bytes of run k not merged yet,
// avail[k] of them landed; final_run[k]: the window holds the rest of run k. F1 over the landed
// prefixes (a record cut by the prefix end is not counted) gives each window's complete records; the
// bound is the least key among the last complete records of the non-final windows (every record
// below it has landed in every run); split[k] = the first record of window k not below the bound, so
// merging [0, split[k]) of every window emits a key range no later record can precede. No bound when
// every window is final (split = complete); all splits 0 when a non-final window has no complete
// record yet.
struct ProgressiveSplit {
  std::vector<int64_t> complete, split;
  bool bounded = false;
  std::string bound;
  double ms = 0;
};
ProgressiveSplit plan_progressive_split(const std::vector<const uint8_t*>& windows, const std::vector<int64_t>& avail,
                                        const std::vector<char>& final_run, int kind, GenericRoundsWs& ws,
                                        hipStream_t s);

}  // namespace gpu
}  // namespace uda
