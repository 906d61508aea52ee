// Device generator of secondary-sort map outputs (variable-length Text keys with long common
// prefixes, `skew` of every map's records in the hot partitions). See secgen.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace uda {
namespace gpu {

struct SecGenPlan {
  int maps = 0, partitions = 0;
  uint64_t seed = 0;
  std::vector<int64_t> nrec;        // [map][partition] records
  std::vector<int64_t> part_bytes;  // [map][partition] bytes incl. the EOF marker
  std::vector<int64_t> mof_off;     // maps + 1: MOF m at [mof_off[m], mof_off[m+1]) of the store (256-aligned)
  std::vector<uint64_t> seeds;      // per run
  int64_t store_bytes() const { return mof_off.empty() ? 0 : mof_off.back(); }
};

// Record counts and exact byte sizes (computed on the current device). Hot partitions: every
// `hot_every`-th (0, hot_every, 2 * hot_every, ...; hot_every <= 0: partition 0 only) shares `skew` of
// every map's records evenly, the other partitions share the rest (a multi-GPU job: reduce task 0 of
// every GPU is the skewed one).
SecGenPlan secgen_plan(int maps, int partitions, int64_t records_per_map, double skew, uint64_t seed,
                       int hot_every = 0);
// Write every MOF into `store` (device, store_bytes() bytes). Synchronizes `s`.
void secgen_write(const SecGenPlan& p, uint8_t* store, hipStream_t s);

}  // namespace gpu
}  // namespace uda
