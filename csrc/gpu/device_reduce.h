// One reduce task's device merge over HBM-resident map-output partitions, delivered to the host
// reducer: the NetMerger online merge (merge_online + merge_do_merging_phase,
// src/Merger/MergeManager.cc:155-193) for partitions that never leave device memory.
//
// Input: K sorted runs in device memory (the provider's HBM partitions, read in place: the RDMA
// WRITE of the reference is replaced by a pointer, or an IPC-mapped pointer across processes).
// FIXED10 (TeraSort-shaped Text records) inputs are merged in key-range rounds so device memory
// stays bounded: a key sample gives Q-1 bounds, every run is split at them on the device, and round
// q merges the q-th slice of every run (F2 -> F3 -> F4) into one of two output slots while the host
// delivers round q-1: SDMA pieces into a pinned ring, cut into <= kv_buf whole-record buffers handed
// to the sink, the last one carrying the IFile EOF marker.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "kernels.h"

namespace uda {
namespace gpu {

struct DeviceReduceConfig {
  int device = 0;
  int64_t kv_buf_bytes = 1 << 20;
  int64_t round_bytes = 2ll << 30;    // target merged bytes per round (two output slots of this size)
  int64_t piece_bytes = 64ll << 20;   // D2H granule
  int pinned_slots = 4;
  int64_t sample_every = 4096;        // one key sampled per this many records for the round bounds
  // HBM admission (hbm_ledger.h): the task's round working set is reserved before its merge; a
  // round that could never fit the budget is halved until it does. A reservation already bound to
  // the calling thread (a caller that reserved for decode + merge at once) is drawn from instead.
  std::function<bool()> stop;         // gives up waiting for HBM when true
  // device_reduce_fixed_blocks: a device-wide turn for each round's block decode (the node's tasks decode
  // one at a time, FIFO: the first rounds reach the link after one decode instead of all of them).
  // decode_turn() returns false when the task stopped while waiting; decode_done() ends the turn.
  std::function<bool()> decode_turn;
  std::function<void()> decode_done;
};

struct DeviceReduceStats {
  int64_t records = 0;
  int64_t bytes = 0;          // record bytes delivered (EOF excluded)
  int64_t buffers = 0;
  int rounds = 0;
  int merge_passes = 0;
  double plan_ms = 0, merge_wait_ms = 0, d2h_wait_ms = 0, sink_ms = 0;
  double hbm_wait_ms = 0;      // waiting for the HBM reservation
  double decode_wait_ms = 0;   // device_reduce_fixed_blocks: waiting for decode turns
  int64_t hbm_reserved = 0;    // bytes reserved for the round working set
  int64_t round_bytes = 0;     // round size used (after any shrink to fit the budget)
  int64_t decoded_blocks = 0;  // device_reduce_fixed_blocks: blocks decoded over all rounds
};

// Build what a FIXED10 task's first round would otherwise build on its critical path (a fresh reduce
// task process: Hadoop runs every reduce task in its own JVM): a pooled workspace with its stream,
// a merger sized for `runs` runs and rounds of `round_bytes` (its upload slots and plan tables; the
// round's output slots stay for the HBM admission), and the delivery ring in the SDMA engine's cache.
// count > 1: that many at once (a node daemon ahead of the concurrent tasks it will host).
void prewarm_device_reduce(const DeviceReduceConfig& cfg, int runs, int count = 1);

// HBM a FIXED10 round working set of `round_bytes` merged bytes needs (two output slots and the
// merger's per-round tables), for admission.
int64_t fixed_round_ws_bytes(int64_t round_bytes, int runs);

// True if every run holds whole TeraSort-shaped records (VInt 11, VInt 91, Text 10 + 90 bytes).
// Synchronizes `s`.
bool runs_are_fixed10(const std::vector<RunDesc>& runs, hipStream_t s);

// Merge `runs` and call sink(buf, len) with every delivery buffer (EOF included in the last).
// A nonzero sink return aborts with an exception.
DeviceReduceStats device_reduce_fixed(const DeviceReduceConfig& cfg, const std::vector<RunDesc>& runs,
                                      const std::function<int(const uint8_t*, int64_t)>& sink);

struct BlockPlan;
// Block-compressed FIXED10 partitions (plan: plan_block_streams_device, every block of every run, dst =
// the run's raw offset + the block's) merged in key-range rounds that decode only the blocks each round
// covers (block first-key index from a prefix decode): device memory is two round inputs and two round
// outputs, not the decoded partitions. *streamed false (nothing delivered): not TeraSort-shaped sorted
// runs; the caller decodes the partitions whole. codec: uda::Codec value.
DeviceReduceStats device_reduce_fixed_blocks(const DeviceReduceConfig& cfg, int codec, const BlockPlan& plan,
                                             const std::function<int(const uint8_t*, int64_t)>& sink,
                                             bool* streamed);

}  // namespace gpu
}  // namespace uda
