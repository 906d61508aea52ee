// Device k-way merge of arbitrary IFile runs (any supported key class, variable-length records).
// Used by the NetMerger's GPU backend (mapred.uda.merge.backend=gpu) and the secondary-sort config.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
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
  // runs: device pointers to IFile streams (records, optionally followed by the EOF marker).
  // Merged records are written to `out` (capacity out_cap). Buffer cuts are chosen so that every
  // delivery buffer holds whole records and at most `kv_buf` bytes (EOF added by the caller).
  // Synchronizes `s` (the record counts size the workspace).
  GenericMergeResult merge(const std::vector<const uint8_t*>& runs, const std::vector<int64_t>& run_bytes,
                           int kind, uint8_t* out, int64_t out_cap, int64_t kv_buf, hipStream_t s);

  // runs the last merge indexed with the serial F1 walk (records longer than the parallel entry table)
  int f1_serial_runs() const { return f1_serial_runs_; }

 private:
  int f1_serial_runs_ = 0;
  void reserve(int64_t records, int runs);
  DeviceBuffer elems_a_, elems_b_, splits_, sizes_, out_off_, scan_tmp_, cuts_, offsets_, tables_, side_, ck_, f1ws_;
  int64_t cap_records_ = 0;
  int cap_runs_ = 0;
};

}  // namespace gpu
}  // namespace uda
