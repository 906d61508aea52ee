// Node-local control plane for the ranks of one job: a POSIX shared-memory segment that every rank
// process maps. It carries what the data plane needs besides the bytes themselves:
//   * a barrier and an abort flag (a failing rank wakes every waiter; a rank whose process died is
//     detected from its pid, so peers throw instead of hanging),
//   * per-rank monotonically increasing counters (round sequence numbers: "my outbox for round k is
//     written", "I finished reading the peers' outboxes of round k", "my copies of round k landed"),
//   * per-rank mailboxes (small all-to-all of int64 counts) and double-buffered outboxes (the slice
//     lists a sender publishes for one exchange round),
//   * per-rank tables of exported device allocations (hipIpc handles as opaque blobs).
//
// Reference analogue: the RDMA-CM connection setup and the SEND/RECV control messages of the
// shuffle (src/DataNet/RDMAClient.cc:215-356 private-data exchange of {qp, credits, rkey};
// RDMAServer.cc:44-136 request parsing; credits as flow control, RDMAComm.cc:707-752). On one
// MI355X node the ranks share DRAM, so the control messages become cache lines in a shared segment
// and the data plane reads peer HBM directly (xGMI).
//
// Pure host code (no HIP): tested on the CPU tier with real processes.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace uda {

class ShmGroup {
 public:
  enum Counter : int { kOut = 0, kIn = 1, kDone = 2, kUser = 3, kCounters = 4 };
  static constexpr int kMaxAllocs = 64;
  static constexpr int kAllocBlob = 64;  // bytes of an exported-allocation handle

  // Rank 0 creates `name` (a leading '/' is added), the others attach (waiting up to timeout_s for
  // it to appear). The constructor is collective: it returns once every rank has attached, and rank
  // 0 then unlinks the name, so nothing is left in /dev/shm even if a rank crashes later.
  ShmGroup(const std::string& name, int rank, int world, size_t mailbox_bytes, size_t outbox_bytes,
           double timeout_s = 900);
  ~ShmGroup();
  ShmGroup(const ShmGroup&) = delete;
  ShmGroup& operator=(const ShmGroup&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }

  // Collective barrier; throws if the group was aborted, a peer died or the timeout passed.
  void barrier(const char* what = "barrier");
  // Same, but gives up after `timeout_s` without aborting the group (teardown).
  bool try_barrier(double timeout_s);
  // Mark the group failed (first reason wins); every waiter of every rank throws.
  void abort(const std::string& why);
  bool aborted() const;
  std::string abort_reason() const;
  // Throw if aborted (cheap).
  void check() const;

  void publish(Counter c, int64_t v);  // release store of this rank's counter
  int64_t read(Counter c, int peer) const;  // acquire load
  // Wait until counter c of `peer` (or of every other rank when peer < 0) is >= v.
  void wait_at_least(Counter c, int peer, int64_t v, const char* what);

  uint8_t* mailbox(int r) const;
  size_t mailbox_bytes() const { return mailbox_bytes_; }
  uint8_t* outbox(int r, int parity) const;
  size_t outbox_bytes() const { return outbox_bytes_; }

  // recv[p*n + i] <- rank p's send[me*n + i] (host memory; chunked through the mailboxes).
  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n);

  // Append an allocation record (blob <= kAllocBlob bytes, plus its size); returns its id.
  int publish_alloc(const void* blob, size_t len, int64_t size);
  // Copy peer's allocation `id` (false if it has not been published yet).
  bool read_alloc(int peer, int id, void* blob, size_t len, int64_t* size) const;

 private:
  struct Header;
  struct RankArea;
  Header* hdr() const;
  RankArea* area(int r) const;
  template <typename Pred>
  void spin_wait(Pred ready, const char* what, double timeout_s, bool abort_on_timeout);
  void check_peers_alive();

  std::string name_;
  int rank_, world_;
  size_t mailbox_bytes_, outbox_bytes_;
  double timeout_s_;
  size_t total_ = 0;
  uint8_t* base_ = nullptr;
  size_t off_ranks_ = 0, off_mail_ = 0, off_out_ = 0;
};

}  // namespace uda
