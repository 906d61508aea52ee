// Node merge service: every reduce task of the node runs its NetMerger inside one long-lived process
// per node -- the node daemon (uda_mof_supplier, started by the provider front end in the NodeManager;
// node_daemon.h) -- and the process Hadoop starts for a reduce task (a YarnChild JVM loading libuda.so)
// is a thin client of it.
//
// Why (MI355X): a fresh process pays the HIP runtime and ROCr start (~330 ms), the library's code
// objects (~70 ms), its workspaces and pinned rings (~90 ms) and hipIpc mappings of the provider's
// HBM before its first merged byte, and 15 such processes starting together contend in the driver.
// The reference runs the NetMerger inside every reduce task JVM (src/UdaBridge.cc:187-263,
// src/Merger/NetMergerMain.cc:44-77), which is cheap for a CPU heap merge over RDMA; for a GPU merge
// the process that holds the GPU context, the pools and the HBM store is the one that should merge.
// The client forwards the host interface 1:1, so the Java side sees no difference:
//   startNative / doCommandNative / reduceExitMsgNative   -> HELLO / CMD / EXIT frames
//   getConfData                                           <- CONF_REQ (answered by the client's host)
//   dataFromUda                                           <- DATA: the merged buffer stays where the
//       service's SDMA engine wrote it (pinned host memory shared with the client through a memfd
//       passed over the socket); the client hands a pointer into its mapping of it to dataFromUda
//       and acknowledges, so no byte is copied on the way
//   fetchOverMessage / failureInUda                       <- FETCH_OVER / FAIL
// A client whose service is unreachable (or that the service refuses) falls back to an in-process
// NetMerger (uda_bridge.cc).
//
// Transport: one Unix stream socket per reduce task (mapred.uda.gpu.merge.service: "auto" =
// "@uda-merge-<data port>" in the abstract namespace, any node-local process can reach it; or a path).
// Access: the peer's uid (SO_PEERCRED) must be the service's own (the default: YARN without the Linux
// container executor runs every task as the NodeManager's user) or be listed in
// mapred.uda.gpu.merge.service.users (user names / uids, or "*" = any local user), at most
// max.sessions.per.user sessions per foreign uid. A task hosted for a foreign uid is confined
// (reduce_task.h TaskSandbox): its local dirs must lie inside the node's own local directories
// (mapred.uda.gpu.merge.service.local.dirs, default yarn.nodemanager.local-dirs / mapred.local.dir), its id
// may not name a path, and it reads back / unlinks only files this process's user wrote. The client
// checks the service's uid the same way (the service's own or root, or
// mapred.uda.gpu.merge.service.server.users), so a process squatting the abstract name never sees a
// task's configuration or feeds it records. A session whose
// client disappears stops its task; a client whose service disappears reports a failure to its host
// (Hadoop then falls back to its vanilla shuffle). A hung client cannot hold up the others: every
// connection's HELLO is read on a thread of its own, and a configuration pull it does not answer
// within conf.timeout ends its session.
#pragma once
#include <sys/types.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "uda/host.h"

namespace uda {

class MergeService {
 public:
  struct Options {
    std::string path;          // socket path or "@abstract-name"; "" = no listener (connections come by adopt())
    std::string users;         // allowed client users besides our own: "*", or user names / uids separated by ','
    int max_sessions = 256;    // live hosted tasks; more are refused (the client merges in its own process)
    int max_sessions_per_user = 64;  // live hosted tasks of one foreign uid
    std::vector<std::string> local_roots;  // canonical directories a foreign uid's task may use
    int force_device = -1;     // >= 0: every hosted task merges on this HIP device (a per-GPU node daemon)
    // a session is over (its task finished or it was refused): its HELLO token (a router's bookkeeping)
    std::function<void(uint64_t token)> session_closed;
    double conf_timeout_s = 60;
    double hello_timeout_s = 10;
    // a hosted task ended (its session is over): e.g. drop the references its descriptors hold in the
    // HBM store living in this process, whether or not the task released them itself
    std::function<void(const std::string& reduce_task_id)> session_ended;
    // defaults of this host for keys a hosted task reads: sent as the default of the configuration pull,
    // so the client's own value (a key its job sets) still wins
    std::map<std::string, std::string> conf_defaults;
  };
  // Listen on `path` (a stale socket file is replaced). Pinned host memory allocated by this process
  // from now on is shareable with clients (sdma.h set_pinned_shareable).
  explicit MergeService(const std::string& path);
  explicit MergeService(const Options& o);
  ~MergeService();  // stops accepting, stops every session's task, joins
  MergeService(const MergeService&) = delete;
  MergeService& operator=(const MergeService&) = delete;
  const std::string& path() const { return opt_.path; }
  // A client connection accepted elsewhere (a router that passed its descriptor over SCM_RIGHTS): handled
  // as if this service had accepted it. Takes ownership of fd. Queued for the acceptor thread, which
  // starts its handshake: the caller (the node daemon's control channel) never creates a thread or
  // waits for mu_, and with them for the process's address-space lock that thread creation takes.
  void adopt(int fd);
  int64_t sessions() const { return sessions_.load(); }
  int64_t refused() const { return refused_.load(); }
  int64_t zero_copy_buffers() const { return zero_copy_.load(); }
  int64_t bounced_buffers() const { return bounced_.load(); }
  std::string stats_json() const;
  // "auto" -> the node's default name for the provider on `data_port`
  static std::string default_path(int data_port);
  // true when `uid` may use the service under `users` (the service's own uid always may)
  static bool user_allowed(const std::string& users, uid_t uid);

  struct Session;

 private:
  void accept_main();
  void handshake(int fd);  // on a thread per connection: credentials, HELLO, session start
  void start_handshake(int fd);  // on the acceptor thread
  Options opt_;
  int listen_fd_ = -1;
  int wake_fd_ = -1;  // eventfd: adopt() wakes the acceptor
  std::mutex aq_mu_;
  std::vector<int> adopted_;  // descriptors adopt() queued for the acceptor
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::condition_variable sess_cv_;  // a session was registered (a data connection waits for its owner)
  std::vector<std::shared_ptr<Session>> live_;
  std::map<uint64_t, std::thread> shakes_;  // handshake threads (by a sequence number)
  std::set<uint64_t> shakes_done_;
  uint64_t next_shake_ = 0;
  std::atomic<int64_t> sessions_{0}, refused_{0};
  std::atomic<int64_t> zero_copy_{0}, bounced_{0};
  friend struct Session;
};

// One reduce task whose NetMerger runs in the node's merge service.
class RemoteReduceTask {
 public:
  // Connect to the service at `path` and start the task with the startNative arguments. Throws
  // UdaError when the service cannot be reached or refuses the task.
  RemoteReduceTask(const std::string& path, const std::vector<std::string>& args, Host* host);
  ~RemoteReduceTask();
  RemoteReduceTask(const RemoteReduceTask&) = delete;
  RemoteReduceTask& operator=(const RemoteReduceTask&) = delete;
  // INIT / FETCH / FINAL command string; throws UdaError with the service's error.
  void handle(const std::string& cmd);
  // Reduce task close: the service stops and joins the task; its stats are kept for stats_json().
  void exit();
  std::string stats_json();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

}  // namespace uda
