// Host planning of the F3 merge tree: the pairwise passes that turn S sorted segments (grouped by
// reducer) into one sorted segment per group. Shared by the FIXED10 (TeraSort) and GENERIC mergers.
//
// Reference role: the PriorityQueue over all segments of one reduce task
// (src/Merger/MergeQueue.h:238-269,299-321); with several reduce tasks per GPU each group is one
// reduce task's queue, and groups never exchange records.
#pragma once
#include <cstdint>
#include <vector>

#include "kernels.h"

namespace uda {
namespace gpu {

struct MergePassPlan {
  std::vector<int64_t> pairs;        // 3 per pair: a0, a1 (= b0), b1
  std::vector<int64_t> tile_prefix;  // npairs + 1
  int npairs = 0;
  int ntiles = 0;
};

// seg: element offsets of the S segments (S+1 ascending entries). group_first: index of the first
// segment of every group plus a final S (G+1 entries; groups may be empty). Every pass moves every
// element (ping-pong buffers), so single segments are copied through as pairs with an empty B.
// Returns no passes when every group already holds at most one segment.
inline std::vector<MergePassPlan> plan_merge_passes(std::vector<int64_t> seg, std::vector<int> group_first,
                                                    int64_t tile = kMergeTile) {
  std::vector<MergePassPlan> passes;
  auto more = [&] {
    for (size_t g = 0; g + 1 < group_first.size(); ++g)
      if (group_first[g + 1] - group_first[g] > 1) return true;
    return false;
  };
  while (more()) {
    MergePassPlan p;
    p.tile_prefix.push_back(0);
    std::vector<int64_t> nseg{seg[0]};
    std::vector<int> ngroup{0};
    for (size_t g = 0; g + 1 < group_first.size(); ++g) {
      const int s0 = group_first[g], s1 = group_first[g + 1];
      for (int s = s0; s < s1; s += 2) {
        const int64_t a0 = seg[s], a1 = seg[s + 1];
        const int64_t b1 = (s + 1 < s1) ? seg[s + 2] : a1;
        p.pairs.insert(p.pairs.end(), {a0, a1, b1});
        p.tile_prefix.push_back(p.tile_prefix.back() + (b1 - a0 + tile - 1) / tile);
        nseg.push_back(b1);
      }
      ngroup.push_back((int)nseg.size() - 1);
    }
    p.npairs = (int)p.pairs.size() / 3;
    p.ntiles = (int)p.tile_prefix.back();
    passes.push_back(std::move(p));
    seg.swap(nseg);
    group_first.swap(ngroup);
  }
  return passes;
}

}  // namespace gpu
}  // namespace uda
