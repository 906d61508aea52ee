// TeraSort driven only through the UdaBridge C ABI (uda_start / INIT / FETCH / reduce_exit and the
// dataFromUda callback), with HBM-resident map outputs: the integration the plugin layer uses,
// measured end to end. One process per GPU (world = 1: loopback transport inside the process):
//   * map phase stand-in: `maps` MOFs with `reducers` total-order partitions each are generated in
//     HBM (ShuffleJob's TeraGen kernel) and registered with a MOFSupplier handle as device MOFs;
//   * one step = `reducers` reduce tasks, each its own NetMerger handle (one per ReduceTask JVM in
//     Hadoop), started concurrently: INIT, one FETCH per map, then the task merges its partitions
//     in the provider's HBM (descriptor fetch) and streams whole-record buffers to dataFromUda;
//   * dataFromUda is the J2C consumer (KVBuf copy + VInt walk, J2CSink), record counts per reducer
//     are checked every step, key order as well when `validate`.
// world > 1 (one process per GPU, the Hadoop node shape): every rank runs its own MOFSupplier on a
// TCP port with its maps' outputs in its HBM, and `reducers` reduce tasks whose INIT names every
// rank's maps; each task FETCHes its partition of every map from the rank that holds it. The
// answers are device descriptors: a provider in another process is mapped with hipIpcOpenMemHandle
// (peer access: on a multi-GPU node the merge reads the other GPUs' HBM over xGMI), so the map
// outputs never cross PCIe and only the merged records go to the host.
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
class DeviceBuffer;

struct ApiBenchConfig {
  int device = 0;
  int maps = 32;
  int reducers = 8;
  int64_t records_per_map = 1 << 20;
  uint64_t seed = 0x5eed;
  int64_t kv_buf_bytes = 1 << 20;
  int64_t round_bytes = 2ll << 30;   // mapred.uda.gpu.round.bytes of every reduce task
  std::string job = "job_202610160000_0001";
  int rank = 0;                      // this process's rank (world > 1: one per GPU)
  int world = 1;
  int port = 0;                      // world > 1: the TCP port of every rank's MOFSupplier
  std::string bind_addr;             // world > 1: this rank's provider address (127.0.0.<rank + 1>)
  bool host_mofs = false;            // register the MOFs from host memory (fetched as bytes, staged to HBM)
  std::string fetch = "device";      // mapred.uda.gpu.fetch of the reduce tasks: device | host | auto
  int provider_workers = -1;         // mapred.uda.provider.workers (-1 = default)
  int max_concurrent_merges = -1;    // mapred.uda.gpu.max.concurrent.merges (staged path; 0 = no limit, -1 = default)
  std::string transport = "loopback";
  // Hadoop-written MOFs: each map output is written as a file under mof_dir and found by the provider
  // through getPathUda (no registration); the provider's HBM store (provider_hbm_bytes > 0) loads a
  // file into HBM on first touch and answers descriptor fetches from it
  std::string mof_dir;
  bool keep_mof_files = false;       // leave the files (and their directories) behind (a map phase of its own)
  bool start_provider = true;        // false: write the map outputs only (no MOFSupplier in this process)
  int64_t provider_hbm_bytes = 0;
  // "terasort" or "secondary": variable-length Text keys with long common prefixes, `skew` of every
  // map's records in reduce task 0 of every rank (BASELINE config #5; device generator secgen.h)
  std::string workload = "terasort";
  double skew = 0.6;
  // "snappy" / "lzo": every partition is block-compressed (256 KiB blocks) at setup and the compressed
  // MOFs are registered in HBM; INIT announces the codec, so reduce tasks decode on the device (F6)
  std::string codec;
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
  // world > 1: records this rank's maps hold for each of the world * reducers reduce tasks (summed
  // over the ranks by the caller), the expected counts of this rank's tasks, and every rank's
  // provider address ("host:port", by rank).
  std::vector<int64_t> local_partition_records() const;
  void set_expected(const std::vector<int64_t>& e) { expected_ = e; }
  void set_peers(const std::vector<std::string>& hosts) { peers_ = hosts; }
  // The commands reduce task r's host sends (its ReduceTask JVM): INIT, then one FETCH per map, in
  // the order step() issues them. Node mode (bench.py --api --node) feeds them to reduce task
  // processes of their own (uda_reduce_task).
  std::vector<std::string> task_commands(int r) const;
  // TCP port the MOFSupplier listens on (transport tcp), else -1.
  int provider_port() const;

 private:
  ApiBenchConfig cfg_;
  std::unique_ptr<ShuffleJob> gen_;
  void* provider_ = nullptr;  // uda_handle*
  std::vector<int64_t> expected_;
  std::vector<std::string> map_ids_;
  std::vector<std::string> peers_;
  std::vector<std::vector<uint8_t>> host_mofs_;  // host_mofs: the MOFs' bytes in host memory
  std::unique_ptr<DeviceBuffer> sec_store_;  // secondary workload: the MOFs in HBM
  int64_t sec_store_bytes_ = 0;
  std::vector<int64_t> sec_part_records_;  // secondary workload: this rank's maps' records per partition
  std::string map_id(int global_map) const;
  void setup_secondary();
  void compress_store();
  std::unique_ptr<DeviceBuffer> comp_store_;  // codec: the compressed MOFs in HBM
  int64_t comp_bytes_ = 0;

 public:
  int64_t compressed_bytes() const { return comp_bytes_; }

 private:

 public:
  // getPathUda of the provider (mof_dir mode)
  bool resolve(const std::string& map, int reduce, int64_t rec[3], std::string* path) const;
  std::string provider_stats() const;

 private:
  std::map<std::string, std::vector<int64_t>> file_index_;  // map id -> 3 int64 per partition
  std::map<std::string, std::string> file_path_;
  void* provider_ctx_ = nullptr;
};

}  // namespace gpu
}  // namespace uda
