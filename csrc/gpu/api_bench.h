// TeraSort driven only through the UdaBridge C ABI (uda_start / INIT / FETCH / reduce_exit and the
// dataFromUda callback), with HBM-resident map outputs: the integration the plugin layer uses,
// measured end to end. One process, one GPU:
//   * map phase stand-in: `maps` MOFs with `reducers` total-order partitions each are generated in
//     HBM (ShuffleJob's TeraGen kernel) and registered with a MOFSupplier handle as device MOFs;
//   * one step = `reducers` reduce tasks, each its own NetMerger handle (one per ReduceTask JVM in
//     Hadoop), started concurrently: INIT, one FETCH per map, then the task merges its partitions
//     in the provider's HBM (descriptor fetch) and streams whole-record buffers to dataFromUda;
//   * dataFromUda is the J2C consumer (KVBuf copy + VInt walk, J2CSink), record counts per reducer
//     are checked every step, key order as well when `validate`.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace uda {
namespace gpu {

class ShuffleJob;
class J2CSink;

struct ApiBenchConfig {
  int device = 0;
  int maps = 32;
  int reducers = 8;
  int64_t records_per_map = 1 << 20;
  uint64_t seed = 0x5eed;
  int64_t kv_buf_bytes = 1 << 20;
  int64_t round_bytes = 2ll << 30;   // mapred.uda.gpu.round.bytes of every reduce task
  std::string job = "job_202610160000_0001";
};

class ApiTeraSortBench {
 public:
  explicit ApiTeraSortBench(const ApiBenchConfig& cfg);
  ~ApiTeraSortBench();
  void setup();
  // One reduce wave; returns wall_ms, bytes, records, buffers, order_errors (validate only) and the
  // per-task merge path / descriptor counts in `info`.
  std::map<std::string, double> step(bool validate, std::string* info = nullptr);
  std::vector<int64_t> expected_records() const { return expected_; }
  int64_t store_bytes() const;

 private:
  ApiBenchConfig cfg_;
  std::unique_ptr<ShuffleJob> gen_;
  void* provider_ = nullptr;  // uda_handle*
  std::vector<int64_t> expected_;
  std::vector<std::string> map_ids_;
};

}  // namespace gpu
}  // namespace uda
