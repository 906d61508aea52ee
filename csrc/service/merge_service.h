// Node merge service: every reduce task of the node runs its NetMerger inside one long-lived process
// per node (the provider process, i.e. the NodeManager aux service), and the process Hadoop starts
// for a reduce task (a YarnChild JVM loading libuda.so) is a thin client of it.
//
// Why (MI355X): a fresh process pays the HIP runtime and ROCr start (~330 ms), the library's code
// objects (~70 ms), its workspaces and pinned rings (~90 ms) and hipIpc mappings of the provider's
// HBM before its first merged byte, and 15 such processes starting together contend in the driver.
// The reference runs the NetMerger inside every reduce task JVM (src/UdaBridge.cc:187-263,
// src/Merger/NetMergerMain.cc:44-77), which is cheap for a CPU heap merge over RDMA; for a GPU merge
// the process that holds the GPU context, the pools and the provider's HBM store is the one that
// should merge. The client forwards the host interface 1:1, so the Java side sees no difference:
//   startNative / doCommandNative / reduceExitMsgNative   -> HELLO / CMD / EXIT frames
//   getConfData                                           <- CONF_REQ (answered by the client's host)
//   dataFromUda                                           <- DATA: the merged buffer stays where the
//       service's SDMA engine wrote it (pinned host memory shared with the client through a memfd
//       passed over the socket); the client hands a pointer into its mapping of it to dataFromUda
//       and acknowledges, so no byte is copied on the way
//   fetchOverMessage / failureInUda                       <- FETCH_OVER / FAIL
// A client whose service is unreachable falls back to an in-process NetMerger (uda_bridge.cc).
//
// Transport: one Unix stream socket per reduce task (path: mapred.uda.gpu.merge.service). A service
// session whose client disappears stops its task; a client whose service disappears reports a
// failure to its host (Hadoop then falls back to its vanilla shuffle).
#pragma once
#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "uda/host.h"

namespace uda {

class MergeService {
 public:
  // Listen on `path` (a stale socket file is replaced). Pinned host memory allocated by this process
  // from now on is shareable with clients (sdma.h set_pinned_shareable).
  explicit MergeService(const std::string& path);
  ~MergeService();  // stops accepting, stops every session's task, joins
  MergeService(const MergeService&) = delete;
  MergeService& operator=(const MergeService&) = delete;
  const std::string& path() const { return path_; }
  int64_t sessions() const { return sessions_.load(); }
  int64_t zero_copy_buffers() const { return zero_copy_.load(); }
  int64_t bounced_buffers() const { return bounced_.load(); }

  struct Session;

 private:
  void accept_main();
  std::string path_;
  int listen_fd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::vector<std::shared_ptr<Session>> live_;
  std::atomic<int64_t> sessions_{0};
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
