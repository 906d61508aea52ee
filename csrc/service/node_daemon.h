// The node daemon: the process that holds a node's GPU state for UDA -- the provider's HBM store of map
// output files and the merge service hosting the node's reduce tasks' NetMergers -- started and
// supervised by the provider front end (the MOFSupplier inside the NodeManager's aux service, or the
// TaskTracker).
//
// Reference shape: the MOFSupplier runs inside the NodeManager / TaskTracker JVM
// (src/MOFServer/MOFSupplierMain.cc:87-143) and each NetMerger inside its ReduceTask JVM, so a native
// failure of one reducer falls back for that reducer only (src/UdaBridge.cc:506-530,
// UdaShuffleConsumerPluginShared.java:205-232) and never reaches the NodeManager.
//
// MI355X design: the GPU work of a node -- HBM store loads, hosted merges -- wants one warm process per
// node (one HIP context, the pools, no per-task hipIpc mappings: merge_service.h), but a GPU fault there
// must not take the NodeManager down. So the front end keeps what the reference's MOFSupplier does
// (TCP listener, getPathUda resolution, byte fetches read from the MOF files) and never touches a GPU;
// the daemon is a child process of it (uda_amd/bin/uda_mof_supplier --daemon-fd N) reached over a
// socket pair:
//   front end -> daemon: START (startNative args, data port), ACQUIRE (a descriptor fetch of a resolved
//                        MOF file: job, path, holder, partition offset/length), RELEASE, RELEASE_HOLDER,
//                        JOB_OVER, STATS, EXIT
//   daemon -> front end: READY / FAILED, ACQUIRED (descriptor or decline), CONF_REQ (getConfData of the
//                        NodeManager's configuration), LOG (into the NodeManager's log), STATS_REPLY
// Failure containment:
//   * an error inside one hosted task fails that task only (its client reports failureInUda);
//   * a daemon that dies (a GPU fault, an abort, the OOM killer) fails the hosted tasks of that moment
//     (their clients see the session gone) and nothing else: the front end declines descriptor fetches
//     (reducers fetch the bytes it serves from the MOF files), restarts the daemon (up to
//     mapred.uda.daemon.restarts times), and keeps serving;
//   * the daemon exits when the front end goes away (control socket EOF).
#pragma once
#include <sys/types.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../provider/device_store.h"
#include "uda/host.h"

namespace uda {

class NodeDaemonClient : public DeviceStore {
 public:
  struct Options {
    std::string exe;                       // daemon executable; "" = uda_mof_supplier next to libuda.so
    std::vector<std::string> start_args;   // the provider's startNative arguments
    int data_port = 0;                     // the front end's TCP port (names the merge service socket)
    double start_timeout_s = 120;          // READY within this (a fresh HIP runtime start included)
    int max_restarts = 3;                  // restarts after the daemon died (0: none)
    std::string log_path;                  // the daemon's stderr ("" = /dev/null; its log goes to LOG frames)
    int device = -1;                       // >= 0: a per-GPU daemon (store, hosted tasks and prewarm on it)
    int ndaemons = 1;                      // daemons of the node (the first wave's prewarm is split over them)
  };
  // Spawn the daemon and wait for its READY (or FAILED). Never throws: a daemon that cannot start leaves
  // a client that declines every fetch (ready() false, why() says what happened).
  NodeDaemonClient(const Options& o, Host* host);
  ~NodeDaemonClient() override;  // EXIT, waits for the daemon (then kills it)

  bool ready() const { return ready_.load(); }
  std::string why() const;
  pid_t pid() const { return pid_.load(); }
  int restarts() const { return restarts_.load(); }
  std::string service_path() const;
  // Wait until the daemon is ready (after a restart), up to `s` seconds.
  bool wait_ready(double s);

  bool acquire(const std::string& job, const std::string& path, const std::string& holder, int64_t offset,
               int64_t len, Done done, std::string* why) override;
  void release(const std::string& path, const std::string& holder) override;
  void release_holder(const std::string& job, const std::string& holder) override;
  void job_over(const std::string& job) override;
  std::string stats_json() override;
  // Hand a merge-service client connection (accepted by the front end's router) to the daemon's
  // service; `token` (its HELLO token, 0 for a data connection) counts as a live session until the
  // daemon reports it over. false: the daemon is not ready (the caller keeps fd).
  bool adopt(int fd, uint64_t token);
  int live_sessions() const;
  int device() const { return opt_.device; }

  // The daemon executable next to the loaded libuda.so ("" if none is found).
  static std::string default_exe();
  // The node has a GPU driver (/dev/kfd): "auto" starts a daemon. Checked without initialising HIP in
  // this (the NodeManager's) process.
  static bool node_has_gpu();

 private:
  bool spawn();                 // mu_ NOT held
  void reader_main(int fd, uint64_t gen);
  bool send(uint32_t type, const std::string& payload);
  void daemon_gone(uint64_t gen, const std::string& why);

  Options opt_;
  Host* host_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  int fd_ = -1;                 // control socket (the front end's end)
  uint64_t gen_ = 0;            // daemon generation (restarts)
  std::atomic<pid_t> pid_{0};
  std::atomic<bool> ready_{false};
  std::atomic<bool> stopping_{false};
  std::atomic<int> restarts_{0};
  bool failed_start_ = false;
  std::string why_ = "node daemon not started";
  std::string service_path_;
  int64_t store_bytes_ = 0;
  uint64_t next_id_ = 1;
  std::map<uint64_t, Done> pending_;
  std::map<uint64_t, std::string> stats_replies_;
  std::set<uint64_t> sessions_;  // routed HELLO tokens whose sessions are live
  std::thread reader_;
  std::vector<std::thread> old_readers_;
  std::mutex send_mu_;
};

// One node daemon per GPU (mapred.uda.daemon.per.gpu, default on): daemon i holds GPU i's share of the
// HBM store (MOF files by a hash of their path) and hosts the reduce tasks merging on GPU i, with its own
// HIP context and hardware queues. A fault on one GPU then fails that GPU's hosted tasks only; the other
// daemons keep serving and the dead one is restarted (its NodeDaemonClient supervises it).
// The node's merge-service name (@uda-merge-<port>) is the front end's: a router thread accepts each
// client connection, peeks its first frame (HELLO / DATA_HELLO + the session token) and passes the
// socket (SCM_RIGHTS) to the daemon of the GPU with the fewest live hosted tasks -- a task's data
// connection to the same daemon as its control one. The client is unchanged (merge_service.h); the
// daemon checks the client's credentials on the passed socket as if it had accepted it.
class NodeDaemonSet : public DeviceStore {
 public:
  struct Options {
    NodeDaemonClient::Options daemon;
    int count = 1;             // daemons (one per GPU)
    bool per_gpu = true;       // count 1 included: the daemon is GPU 0's and the front end routes
    std::string service_path;  // the node's merge-service name ("" = none)
  };
  NodeDaemonSet(const Options& o, Host* host);
  ~NodeDaemonSet() override;
  size_t size() const { return d_.size(); }
  NodeDaemonClient& daemon(size_t i) { return *d_.at(i); }
  bool ready() const {
    for (auto& d : d_)
      if (d && d->ready()) return true;
    return false;
  }

  bool acquire(const std::string& job, const std::string& path, const std::string& holder, int64_t offset,
               int64_t len, Done done, std::string* why) override;
  void release(const std::string& path, const std::string& holder) override;
  void release_holder(const std::string& job, const std::string& holder) override;
  void job_over(const std::string& job) override;
  std::string stats_json() override;

  // GPUs of the node (KFD topology; HIP_VISIBLE_DEVICES honoured), without initialising HIP.
  static int node_gpu_count();

 private:
  void route_main();
  size_t store_of(const std::string& path);
  std::mutex route_mu_;
  std::map<std::string, size_t> route_;  // MOF path -> the daemon whose store holds it
  Options opt_;
  std::vector<std::unique_ptr<NodeDaemonClient>> d_;
  int listen_fd_ = -1;
  std::thread router_;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> routed_{0}, refused_{0};
};

// The daemon's main (uda_mof_supplier --daemon-fd N): serve the front end on `ctl_fd` until it says EXIT
// or goes away. Returns the process exit code.
int run_node_daemon(int ctl_fd);

}  // namespace uda
