// MOFSupplier: serves map-output-file partitions to reducers.
//
// Parity:
//   MOFSupplier_main / mof_downcall_handler   (src/MOFServer/MOFSupplierMain.cc:37-157)
//   OutputServer request queue                 (src/MOFServer/MOFServlet.cc:99-180)
//   DataEngine: index resolution via getPathUda on first touch, refcounted fd cache, aligned
//   O_DIRECT AIO chunk reads, completion -> data + ACK (src/MOFServer/IndexInfo.cc:141-376)
// MI355X-native differences: partitions can be registered from memory (host or, through the GPU
// engine, HBM) and the disk path goes through io_uring (uda/aio.h). The data lands directly in the
// transport's destination buffer (the one-sided RDMA WRITE analogue) instead of a staging chunk.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "uda/aio.h"
#include "uda/cmd.h"
#include "uda/host.h"
#include "uda/transport.h"
#include "device_store.h"

namespace uda {

class Supplier : public DataServer {
 public:
  struct Options {
    int workers = 8;             // DataEngine threads (mapred.uda.provider.workers)
    int io_threads = 4;          // AsyncIO pool size (blocked.threads.per.disk analogue)
    bool odirect = false;        // read MOF files with O_DIRECT (4 KiB aligned bounce chunks)
    bool copy_serve = false;     // mapred.uda.provider.copy.serve: no by-reference answers (A/B of serve_ref)
    int max_open_files = 512;    // fd cache bound (rlimit analogue)
    std::string transport = "loopback";  // loopback | tcp
    std::string loopback_host = "*";
    std::string bind_addr;       // tcp: listen address (mapred.uda.provider.bind.address; empty = any)
  };
  Supplier(const NetlevOptions& net, const Options& o, Host* host);
  ~Supplier() override;
  // HBM store for file MOFs (device_store.h): descriptor fetches of MOFs found through getPathUda are
  // answered with device descriptors of the file's copy in HBM (loaded on first touch). Set before
  // start() or later (a node daemon is started once the listener has its port); none: such fetches are
  // declined (the reducer fetches the bytes).
  void set_store(std::shared_ptr<DeviceStore> store) {
    std::lock_guard<std::mutex> g(store_mu_);
    store_ = std::move(store);
  }
  std::shared_ptr<DeviceStore> store() {
    std::lock_guard<std::mutex> g(store_mu_);
    return store_;
  }
  void start();
  void stop();

  // In-memory MOF registration: index[p] = {start_offset, raw_length, part_length}. device >= 0:
  // `data` is device memory of that HIP device (an HBM-resident MOF): descriptor fetches get its
  // address / IPC handle instead of bytes, byte fetches are served by a device-to-host copy.
  void register_mof(const std::string& job, const std::string& map, const uint8_t* data, int64_t len,
                    std::vector<IndexRec> index, int device = -1);
  void serve(const FetchRequest& req, uint8_t* dst, FetchDone done) override;
  // Byte fetches by reference (the TCP transport's zero-copy send): host-memory MOFs as they lie, MOF
  // files as a file range (sendfile); HBM MOFs and O_DIRECT reads through a chunk of this request's own.
  bool serve_ref(const FetchRequest& req, RefDone done) override;

  int port() const { return server_ ? server_->port() : -1; }
  int64_t requests() const { return requests_.load(); }
  int64_t bytes_served() const { return bytes_.load(); }
  int64_t descriptors_served() const { return descriptors_.load(); }
  // CLOCK_BOOTTIME ms of the first descriptor request (0: none yet): the fetch chain's place on a timeline
  double first_descriptor_request_boot_ms() const { return first_desc_boot_ms_.load(); }
  // JOB_OVER: the job's MOFs held in the HBM store may be freed.
  void job_over(const std::string& job);
  // {"loads":..,"hits":..,...} of the HBM store ("{}" when there is none)
  std::string hbm_stats_json();
  const char* io_backend() const { return aio_ ? aio_->backend() : "none"; }

 private:
  struct Job {
    FetchRequest req;
    uint8_t* dst;
    FetchDone done;
    RefDone ref_done;  // serve_ref: answer by reference (dst and done unused)
  };
  struct MemMof {
    const uint8_t* data;
    int64_t len;
    std::vector<IndexRec> index;
    int device = -1;
    std::string ipc_handle;           // device MOFs: IPC handle (hex) of the containing allocation
    const uint8_t* ipc_base = nullptr;
  };
  struct OpenFile {
    int fd = -1;
    int refs = 0;
    uint64_t last_use = 0;
  };
  void worker();
  void process(Job& j);
  void process_ref(Job& j);
  bool resolve(const FetchRequest& req, IndexRec* rec, const MemMof** mem);
  int acquire_fd(const std::string& path);
  void release_fd(const std::string& path);

  NetlevOptions net_;
  Options opt_;
  Host* host_;
  std::unique_ptr<AsyncIO> aio_;
  std::unique_ptr<ServerTransport> server_;
  std::mutex store_mu_;
  std::shared_ptr<DeviceStore> store_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  std::vector<std::thread> workers_;
  bool stop_ = false;
  std::mutex idx_mu_;
  std::map<std::string, MemMof> mem_;                    // key job|map
  std::unordered_map<std::string, IndexRec> idx_cache_;  // key job|map|reduce
  std::mutex fd_mu_;
  std::unordered_map<std::string, OpenFile> fds_;
  uint64_t fd_clock_ = 0;
  std::atomic<int64_t> requests_{0}, bytes_{0}, descriptors_{0}, releases_{0};
  std::atomic<double> first_desc_boot_ms_{0};
};

}  // namespace uda
