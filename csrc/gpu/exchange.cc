#include "exchange.h"
#include "device_ptr.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "device_engine.h"
#include "uda/shm_group.h"

namespace uda {
namespace gpu {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r) + " in " + what);
}
#define NCCL_CHECK(x) nccl_check((x), #x)

bool env_flag(const char* name, bool dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atoi(v) != 0;
}

// ------------------------------------------------------------------------------------ RCCL
class RcclExchange : public Exchange {
 public:
  RcclExchange(int rank, int world, const std::string& uid) : rank_(rank), world_(world) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
    if (const char* t = std::getenv("UDA_RCCL_TIMEOUT_S")) timeout_ = std::chrono::seconds(std::max(1, std::atoi(t)));
    pack_ = env_flag("UDA_RCCL_PACK", false);
    descs_.resize(4);
    for (auto& d : descs_) HIP_CHECK(hipEventCreateWithFlags(&d.uploaded, hipEventDisableTiming));
  }
  ~RcclExchange() override {
    if (comm_) (aborted_ ? ncclCommAbort(comm_) : ncclCommDestroy(comm_));
    for (auto& d : descs_)
      if (d.uploaded) (void)hipEventDestroy(d.uploaded);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  int comm_ranks() const override {
    int n = 0;
    if (!comm_ || ncclCommCount(comm_, &n) != ncclSuccess) return -1;
    return n;
  }
  std::string name() const override { return pack_ ? "rccl-packed" : "rccl"; }

  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t s) override {
    const size_t bytes = n * (size_t)world_ * 8;
    if (counts_.size() < bytes * 2) counts_.alloc(bytes * 2);
    int64_t* ds = counts_.as<int64_t>();
    int64_t* dr = ds + n * world_;
    HIP_CHECK(hipMemcpyAsync(ds, send, bytes, hipMemcpyHostToDevice, s));
    NCCL_CHECK(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      NCCL_CHECK(ncclSend(ds + p * n, n, ncclInt64, p, comm_, s));
      NCCL_CHECK(ncclRecv(dr + p * n, n, ncclInt64, p, comm_, s));
    }
    NCCL_CHECK(ncclGroupEnd());
    HIP_CHECK(hipMemcpyAsync(recv, dr, bytes, hipMemcpyDeviceToHost, s));
    wait(s);
  }

  void reserve(int64_t bytes) override {
    if (pack_ && (int64_t)staging_.size() < bytes) staging_.alloc((size_t)std::max<int64_t>(bytes, 16));
  }

  void check() override {
    if (aborted_) throw std::runtime_error("RCCL communicator was aborted after an earlier failure");
    ncclResult_t a = ncclSuccess;
    NCCL_CHECK(ncclCommGetAsyncError(comm_, &a));
    if (a != ncclSuccess && a != ncclInProgress) fail(std::string("RCCL asynchronous error: ") + ncclGetErrorString(a));
  }

  void wait(hipStream_t s) override {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      check();
      if (std::chrono::steady_clock::now() - t0 > timeout_)
        fail("RCCL exchange timed out after " + std::to_string(timeout_.count()) + " s (peer lost?)");
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

  void exchange(const std::vector<std::vector<Span>>& send, const std::vector<std::vector<Span>>& recv,
                hipStream_t s) override {
    if (aborted_) throw std::runtime_error("RCCL communicator was aborted after an earlier failure");
    // A rank that gives up here never enters this round's group, while its peers already inside it
    // wait for its sends until the timeout: every failure before or inside the group aborts the
    // communicator (the peers' async-error polling then sees it) instead of only throwing.
    try {
      exchange_group(send, recv, s);
    } catch (const std::exception& e) {
      fail(std::string("RCCL exchange: ") + e.what());
    }
  }

  void exchange_group(const std::vector<std::vector<Span>>& send, const std::vector<std::vector<Span>>& recv,
                      hipStream_t s) {
    if ((int)send.size() != world_ || (int)recv.size() != world_) throw std::runtime_error("exchange: bad peer lists");
    if (!send[rank_].empty() || !recv[rank_].empty()) throw std::runtime_error("exchange: self slices");
    std::vector<Span> one_send(world_, Span{nullptr, 0}), one_recv(world_, Span{nullptr, 0});
    if (pack_) {
      // stage every peer's slices contiguously (rotating peer order) with one batched-copy launch
      DescSlot& ds = descs_[next_desc_];
      next_desc_ = (next_desc_ + 1) % (int)descs_.size();
      if (ds.used) HIP_CHECK(hipEventSynchronize(ds.uploaded));
      size_t nd = 0;
      for (int p = 0; p < world_; ++p) nd += send[p].size();
      if (ds.host.size() < nd * sizeof(CopyDesc)) {
        ds.host.alloc(std::max<size_t>(nd, 64) * sizeof(CopyDesc));
        ds.dev.alloc(std::max<size_t>(nd, 64) * sizeof(CopyDesc));
      }
      ds.used = true;
      CopyDesc* d = ds.host.as<CopyDesc>();
      int n = 0;
      int64_t off = 0, max_bytes = 0;
      for (int k = 1; k < world_; ++k) {
        const int to = (rank_ + k) % world_;
        const int64_t beg = off;
        for (const Span& sp : send[to]) {
          if (off + sp.bytes > (int64_t)staging_.size()) throw std::runtime_error("exchange: staging too small");
          d[n++] = CopyDesc{sp.ptr, staging_.as<uint8_t>() + off, sp.bytes};
          max_bytes = std::max(max_bytes, sp.bytes);
          off += sp.bytes;
        }
        one_send[to] = Span{staging_.as<uint8_t>() + beg, off - beg};
      }
      if (n > 0) {
        HIP_CHECK(hipMemcpyAsync(ds.dev.as(), d, sizeof(CopyDesc) * n, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipEventRecord(ds.uploaded, s));
        launch_batched_copy(ds.dev.as<CopyDesc>(), n, max_bytes, s);
      }
      for (int p = 0; p < world_; ++p) {
        if (p == rank_ || recv[p].empty()) continue;
        int64_t total = 0;
        for (const Span& sp : recv[p]) {
          if (sp.ptr != recv[p][0].ptr + total)
            throw std::runtime_error("exchange: packed mode needs contiguous receive slices per peer");
          total += sp.bytes;
        }
        one_recv[p] = Span{recv[p][0].ptr, total};
      }
    }
    NCCL_CHECK(ncclGroupStart());
    for (int k = 1; k < world_; ++k) {
      const int to = (rank_ + k) % world_;  // rotating order spreads the xGMI link load
      const int from = (rank_ - k + world_) % world_;
      if (pack_) {
        if (one_send[to].bytes > 0)
          NCCL_CHECK(ncclSend(one_send[to].ptr, (size_t)one_send[to].bytes, ncclUint8, to, comm_, s));
        if (one_recv[from].bytes > 0)
          NCCL_CHECK(ncclRecv(const_cast<uint8_t*>(one_recv[from].ptr), (size_t)one_recv[from].bytes, ncclUint8, from,
                              comm_, s));
      } else {
        for (const Span& sp : send[to]) NCCL_CHECK(ncclSend(sp.ptr, (size_t)sp.bytes, ncclUint8, to, comm_, s));
        for (const Span& sp : recv[from])
          NCCL_CHECK(ncclRecv(const_cast<uint8_t*>(sp.ptr), (size_t)sp.bytes, ncclUint8, from, comm_, s));
      }
    }
    NCCL_CHECK(ncclGroupEnd());
  }

 private:
  // A lost peer leaves kernels of this communicator waiting forever: abort it so the device drains,
  // then surface the failure (the bridge turns it into failureInUda / a failed step).
  [[noreturn]] void fail(const std::string& why) {
    if (!aborted_) {
      aborted_ = true;
      (void)ncclCommAbort(comm_);
      comm_ = nullptr;
    }
    throw std::runtime_error(why);
  }
  struct DescSlot {
    PinnedBuffer host;
    DeviceBuffer dev;
    hipEvent_t uploaded = nullptr;
    bool used = false;
  };
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
  bool aborted_ = false;
  bool pack_ = false;
  std::chrono::seconds timeout_{900};
  DeviceBuffer counts_, staging_;
  std::vector<DescSlot> descs_;
  int next_desc_ = 0;
};


// ------------------------------------------------------------------------------------ checks
// The point-to-point rules every backend enforces (exchange.h): a receiver's slice list from a peer
// must pair 1:1 with what the peer sends it, and both ends are device allocations.
void check_pairing(int from, int to, const std::vector<int64_t>& sent_bytes, const std::vector<Span>& recv) {
  if (sent_bytes.size() != recv.size())
    throw std::runtime_error("exchange: rank " + std::to_string(from) + " sends " + std::to_string(sent_bytes.size()) +
                             " slices to rank " + std::to_string(to) + ", which posts " + std::to_string(recv.size()) +
                             " receives (send/recv pairing violated)");
  for (size_t i = 0; i < recv.size(); ++i)
    if (sent_bytes[i] != recv[i].bytes)
      throw std::runtime_error("exchange: slice " + std::to_string(i) + " from rank " + std::to_string(from) + " to " +
                               std::to_string(to) + " is " + std::to_string(sent_bytes[i]) +
                               " bytes, the receive is " + std::to_string(recv[i].bytes));
}

void check_device_memory(const void* p, const char* role) {
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeDevice) {
    (void)hipGetLastError();
    throw std::runtime_error(std::string("exchange: ") + role +
                             " slice is not device memory (host-pinned or unregistered buffers cannot be sent "
                             "peer to peer; stage them into HBM first)");
  }
}

// ------------------------------------------------------------------------------------ local group
// Threads of one process meet at barriers. A rank that fails between barriers aborts the group so
// the others throw instead of waiting forever; the group is erased with its last member.
struct Group {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  bool aborted = false;
  bool failed = false;  // a rank's exchange failed after the entry barrier (see LocalExchange::exchange)
  std::vector<const std::vector<std::vector<Span>>*> sends;  // per rank, valid between barriers
  std::vector<const int64_t*> counts;
  // per rank: event recorded after its receive copies of exchange seq (parity seq & 1), and the
  // number of exchanges whose event was recorded
  std::vector<std::array<hipEvent_t, 2>> done_ev;
  std::vector<int64_t> done_seq;
  // per rank: event recorded on its stream when it entered the exchange: its send slices are
  // written once the stream passed it (receivers' streams wait for it before pulling)
  std::vector<hipEvent_t> ready_ev;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw std::runtime_error("local exchange group aborted by another rank");
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen || aborted; });
      if (aborted) throw std::runtime_error("local exchange group aborted by another rank");
    }
  }
  void abort() {
    std::lock_guard<std::mutex> g(mu);
    aborted = true;
    cv.notify_all();
  }
};

std::mutex g_groups_mu;
std::map<std::string, std::shared_ptr<Group>> g_groups;

class LocalExchange : public Exchange {
 public:
  LocalExchange(const std::string& name, int rank, int world) : name_(name), rank_(rank), world_(world) {
    std::lock_guard<std::mutex> g(g_groups_mu);
    auto& grp = g_groups[name];
    if (!grp || grp->aborted) {
      grp = std::make_shared<Group>();
      grp->world = world;
      grp->sends.assign(world, nullptr);
      grp->counts.assign(world, nullptr);
      grp->done_ev.assign(world, {nullptr, nullptr});
      grp->done_seq.assign(world, 0);
      grp->ready_ev.assign(world, nullptr);
    }
    if (grp->world != world) throw std::runtime_error("local exchange: world mismatch");
    group_ = grp;
    std::lock_guard<std::mutex> gl(grp->mu);
    for (auto& e : grp->done_ev[rank]) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&grp->ready_ev[rank], hipEventDisableTiming));
    grp->done_seq[rank] = 0;
  }
  ~LocalExchange() override {
    {
      std::lock_guard<std::mutex> gl(group_->mu);
      for (auto& e : group_->done_ev[rank_])
        if (e) (void)hipEventDestroy(e), e = nullptr;
      if (group_->ready_ev[rank_]) (void)hipEventDestroy(group_->ready_ev[rank_]), group_->ready_ev[rank_] = nullptr;
    }
    std::lock_guard<std::mutex> g(g_groups_mu);
    auto it = g_groups.find(name_);
    if (it != g_groups.end() && it->second == group_ && group_.use_count() <= 2) g_groups.erase(it);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  std::string name() const override { return "local"; }

  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t) override {
    Group& g = *group_;
    g.counts[rank_] = send;
    g.barrier();
    for (int p = 0; p < world_; ++p) std::memcpy(recv + p * n, g.counts[p] + (size_t)rank_ * n, n * 8);
    g.barrier();
  }

  void exchange(const std::vector<std::vector<Span>>& send, const std::vector<std::vector<Span>>& recv,
                hipStream_t s) override {
    Group& g = *group_;
    // a rank that throws before the barrier must wake its peers (Group::barrier has no timeout)
    if ((int)send.size() != world_ || (int)recv.size() != world_) {
      g.abort();
      throw std::runtime_error("exchange: bad peer lists");
    }
    if (!send[rank_].empty() || !recv[rank_].empty()) {
      g.abort();
      throw std::runtime_error("exchange: self slices");
    }
    const int64_t seq = seq_++;
    g.sends[rank_] = &send;
    HIP_CHECK(hipEventRecord(g.ready_ev[rank_], s));
    g.barrier();
    // Between the two barriers the peers read this rank's send list and enqueue copies from its
    // memory, so a rank that fails here must not return (and free either) before they are done: it
    // marks the group failed and still meets the exit barrier; then every rank drains its copies,
    // meets once more and throws.
    std::string err;
    try {
      for (int k = 1; k < world_; ++k) {
        const int from = (rank_ - k + world_) % world_;
        const auto& theirs = (*g.sends[from])[rank_];
        if (!theirs.empty()) HIP_CHECK(hipStreamWaitEvent(s, g.ready_ev[from], 0));  // sender's writes done
        const auto& mine = recv[from];
        std::vector<int64_t> sizes(theirs.size());
        for (size_t i = 0; i < theirs.size(); ++i) sizes[i] = theirs[i].bytes;
        check_pairing(from, rank_, sizes, mine);
        for (size_t i = 0; i < mine.size(); ++i) {
          check_device_memory(theirs[i].ptr, "send");
          check_device_memory(mine[i].ptr, "receive");
          HIP_CHECK(hipMemcpyAsync(const_cast<uint8_t*>(mine[i].ptr), theirs[i].ptr, (size_t)mine[i].bytes,
                                   hipMemcpyDeviceToDevice, s));
        }
      }
      HIP_CHECK(hipEventRecord(g.done_ev[rank_][seq & 1], s));
      {
        std::lock_guard<std::mutex> gl(g.mu);
        g.done_seq[rank_] = seq + 1;
      }
      g.cv.notify_all();
    } catch (const std::exception& e) {
      err = e.what();
      std::lock_guard<std::mutex> gl(g.mu);
      g.failed = true;
    }
    g.barrier();  // peers' send lists are no longer read
    bool failed;
    {
      std::lock_guard<std::mutex> gl(g.mu);
      failed = g.failed;
    }
    if (failed) {
      (void)hipStreamSynchronize(s);  // copies reading the peers' memory have landed
      try {
        g.barrier();
      } catch (const std::exception&) {  // a peer passed it first and marked the group aborted
      }
      g.abort();  // the group is unusable from here on
      throw std::runtime_error(err.empty() ? "local exchange group aborted by another rank" : err);
    }
  }

  // The peers read this rank's send slices on their own streams: wait for their copies' events.
  void wait_sent(int64_t seq) override {
    Group& g = *group_;
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      hipEvent_t ev;
      {
        std::unique_lock<std::mutex> lk(g.mu);
        g.cv.wait(lk, [&] { return g.done_seq[p] >= seq + 1 || g.aborted; });
        if (g.aborted) throw std::runtime_error("local exchange group aborted by another rank");
        ev = g.done_ev[p][seq & 1];
      }
      HIP_CHECK(hipEventSynchronize(ev));
    }
  }

  void quiesce() override { group_->barrier(); }

 private:
  std::string name_;
  int rank_, world_;
  int64_t seq_ = 0;
  std::shared_ptr<Group> group_;
};

// ------------------------------------------------------------------------------------ IPC
// Rank processes on one node. Per exchange seq k (parity k & 1):
//   1. wait until every peer has read this rank's outbox of exchange k-2 (same parity),
//   2. write the outbox: per destination, (exported allocation id, offset, bytes) of every slice,
//      exporting new allocations over hipIpc on first use; publish kOut = k+1,
//   3. for every source peer (rotating order): wait for its kOut >= k+1, check the pairing against
//      the local receive list, map the peer's allocation (once) and enqueue the pull copy on `s`;
//      publish kIn = k+1,
//   4. a progress thread publishes kDone = k+1 once this rank's copies of exchange k completed,
//      which is what wait_sent(k) of the senders waits for.
class IpcExchange : public Exchange {
  struct Entry {
    int32_t alloc;
    int32_t pad;
    int64_t off;
    int64_t bytes;
  };
  static constexpr size_t kMaxEntries = 65536;

 public:
  IpcExchange(const std::string& name, int rank, int world, int device)
      : rank_(rank),
        world_(world),
        device_(device),
        grp_(name, rank, world, (size_t)256 << 10, 16 + (size_t)8 * world + kMaxEntries * sizeof(Entry),
             env_timeout()) {
    HIP_CHECK(hipSetDevice(device_));
    descs_.resize(4);
    for (auto& d : descs_) HIP_CHECK(hipEventCreateWithFlags(&d.uploaded, hipEventDisableTiming));
    progress_ = std::thread([this] { progress_loop(); });
  }
  ~IpcExchange() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (progress_.joinable()) progress_.join();
    // nobody may still read this rank's memory when its owner frees it
    if (!grp_.aborted()) (void)grp_.try_barrier(60);
    for (auto& kv : mapped_) (void)hipIpcCloseMemHandle(kv.second.first);
    for (auto e : free_ev_) (void)hipEventDestroy(e);
    if (ready_ev_) (void)hipEventDestroy(ready_ev_);
    for (auto& d : descs_)
      if (d.uploaded) (void)hipEventDestroy(d.uploaded);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  std::string name() const override { return "ipc"; }

  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t) override {
    grp_.alltoall_i64(send, recv, n);
  }

  void exchange(const std::vector<std::vector<Span>>& send, const std::vector<std::vector<Span>>& recv,
                hipStream_t s) override {
    const int64_t k = seq_++;
    const int par = (int)(k & 1);
    try {
      if ((int)send.size() != world_ || (int)recv.size() != world_) throw std::runtime_error("exchange: bad peer lists");
      if (!send[rank_].empty() || !recv[rank_].empty()) throw std::runtime_error("exchange: self slices");
      // The peers pull with their own streams: what this rank's stream still has to write into the
      // send slices (staging copies enqueued before this call) must land before the outbox says so.
      bool sends = false;
      for (const auto& v : send) sends = sends || !v.empty();
      if (sends) {
        if (!ready_ev_) HIP_CHECK(hipEventCreateWithFlags(&ready_ev_, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(ready_ev_, s));
        HIP_CHECK(hipEventSynchronize(ready_ev_));
      }
      if (k >= 2) grp_.wait_at_least(ShmGroup::kIn, -1, k - 1, "peers to read the previous outbox");
      uint8_t* ob = grp_.outbox(rank_, par);
      int32_t* cnt = reinterpret_cast<int32_t*>(ob + 16);
      int32_t* first = cnt + world_;
      Entry* e = reinterpret_cast<Entry*>(ob + 16 + (size_t)8 * world_);
      size_t n = 0;
      for (int p = 0; p < world_; ++p) {
        first[p] = (int32_t)n;
        for (const Span& sp : send[p]) {
          if (n >= kMaxEntries) throw std::runtime_error("exchange: too many slices in one round");
          int64_t off = 0;
          const int id = locate(sp.ptr, sp.bytes, &off);
          e[n++] = Entry{id, 0, off, sp.bytes};
        }
        cnt[p] = (int32_t)(n - first[p]);
      }
      reinterpret_cast<int64_t*>(ob)[0] = (int64_t)n;
      grp_.publish(ShmGroup::kOut, k + 1);
      std::vector<CopyDesc> copies;
      int64_t max_bytes = 0;
      for (int kk = 1; kk < world_; ++kk) {
        const int from = (rank_ - kk + world_) % world_;
        grp_.wait_at_least(ShmGroup::kOut, from, k + 1, "a peer's outbox");
        const uint8_t* pb = grp_.outbox(from, par);
        const int32_t* pc = reinterpret_cast<const int32_t*>(pb + 16);
        const int32_t* pf = pc + world_;
        const Entry* pe = reinterpret_cast<const Entry*>(pb + 16 + (size_t)8 * world_) + pf[rank_];
        const int c = pc[rank_];
        std::vector<int64_t> sizes(c);
        for (int i = 0; i < c; ++i) sizes[i] = pe[i].bytes;
        check_pairing(from, rank_, sizes, recv[from]);
        for (int i = 0; i < c; ++i) {
          const uint8_t* src = peer_ptr(from, pe[i].alloc, pe[i].off, pe[i].bytes);
          copies.push_back(CopyDesc{src, const_cast<uint8_t*>(recv[from][i].ptr), pe[i].bytes});
          max_bytes = std::max(max_bytes, pe[i].bytes);
          bytes_pulled_ += pe[i].bytes;
        }
      }
      grp_.publish(ShmGroup::kIn, k + 1);
      if (!copies.empty()) launch_pulls(copies, max_bytes, s);
      hipEvent_t ev = take_event();
      HIP_CHECK(hipEventRecord(ev, s));
      {
        std::lock_guard<std::mutex> g(mu_);
        pending_.push_back({k, ev});
      }
      cv_.notify_all();
    } catch (const std::exception& ex) {
      grp_.abort(std::string("exchange failed: ") + ex.what());
      throw;
    }
  }

  void wait_sent(int64_t seq) override {
    grp_.wait_at_least(ShmGroup::kDone, -1, seq + 1, "peers to finish copying this rank's slices");
  }

  void quiesce() override { grp_.barrier("end of step"); }

  void wait(hipStream_t s) override {
    for (int spin = 0;; ++spin) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      grp_.check();
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

  void check() override {
    grp_.check();
    std::lock_guard<std::mutex> g(mu_);
    if (!progress_error_.empty()) throw std::runtime_error(progress_error_);
  }

 private:
  static double env_timeout() {
    const char* t = std::getenv("UDA_IPC_TIMEOUT_S");
    return t ? std::max(1.0, std::atof(t)) : 900.0;
  }

  // Exported allocation containing [p, p + bytes): its id in this rank's table and the offset.
  int locate(const uint8_t* p, int64_t bytes, int64_t* off) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = exported_.upper_bound(a);
    if (it != exported_.begin()) {
      --it;
      if (a >= it->first && a + (uintptr_t)bytes <= it->first + (uintptr_t)it->second.size) {
        if (!freed_since(reinterpret_cast<const void*>(it->first), it->second.epoch)) {
          *off = (int64_t)(a - it->first);
          return it->second.id;
        }
        // freed and allocated again at the same address: a new export (peers map the new handle)
        exported_.erase(it);
      }
    }
    check_device_memory(p, "send");
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<uint8_t*>(p)) != hipSuccess || !base) {
      (void)hipGetLastError();
      throw std::runtime_error("exchange: send slice is not inside a device allocation");
    }
    if (((uint64_t)size & 0xFFFFFFFFull) >= (1ull << 31))
      throw std::runtime_error("exchange: send allocation of " + std::to_string(size) +
                               " bytes is in the size range whose hipIpc import hangs; allocate it with "
                               "ipc_safe_bytes() (DeviceBuffer does)");
    const uintptr_t b = reinterpret_cast<uintptr_t>(base);
    if (a + (uintptr_t)bytes > b + size) throw std::runtime_error("exchange: send slice crosses its allocation's end");
    hipIpcMemHandle_t h;
    const uint64_t epoch = alloc_epoch();
    HIP_CHECK(hipIpcGetMemHandle(&h, base));
    const int id = grp_.publish_alloc(&h, sizeof(h), (int64_t)size);
    exported_[b] = Exported{size, id, epoch};
    *off = (int64_t)(a - b);
    return id;
  }

  const uint8_t* peer_ptr(int peer, int id, int64_t off, int64_t bytes) {
    const auto key = std::make_pair(peer, id);
    auto it = mapped_.find(key);
    if (it == mapped_.end()) {
      hipIpcMemHandle_t h;
      int64_t size = 0;
      if (!grp_.read_alloc(peer, id, &h, sizeof(h), &size))
        throw std::runtime_error("exchange: rank " + std::to_string(peer) + " named an unpublished allocation");
      void* p = nullptr;
      HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      it = mapped_.emplace(key, std::make_pair(p, size)).first;
    }
    if (off < 0 || bytes < 0 || off + bytes > it->second.second)
      throw std::runtime_error("exchange: slice outside the peer's allocation");
    return static_cast<const uint8_t*>(it->second.first) + off;
  }

  // One launch pulls every slice of the round: the workgroups of all peers' slices run at once, so
  // the reads spread over every xGMI link (per-slice hipMemcpyAsync would serialize them on `s`).
  // Descriptors go through a pinned slot uploaded on `s` (4 slots, reused once their upload landed).
  void launch_pulls(const std::vector<CopyDesc>& copies, int64_t max_bytes, hipStream_t s) {
    DescSlot& ds = descs_[next_desc_];
    next_desc_ = (next_desc_ + 1) % (int)descs_.size();
    if (ds.used) HIP_CHECK(hipEventSynchronize(ds.uploaded));
    const size_t bytes = copies.size() * sizeof(CopyDesc);
    if (ds.host.size() < bytes) {
      ds.host.alloc(std::max<size_t>(bytes, 64 * sizeof(CopyDesc)));
      ds.dev.alloc(std::max<size_t>(bytes, 64 * sizeof(CopyDesc)));
    }
    std::memcpy(ds.host.as(), copies.data(), bytes);
    HIP_CHECK(hipMemcpyAsync(ds.dev.as(), ds.host.as(), bytes, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipEventRecord(ds.uploaded, s));
    ds.used = true;
    for (size_t b = 0; b < copies.size(); b += 65535)  // grid.y limit
      launch_batched_copy(ds.dev.as<CopyDesc>() + b, (int)std::min<size_t>(65535, copies.size() - b), max_bytes, s);
    HIP_CHECK(hipGetLastError());
  }

  hipEvent_t take_event() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_ev_.empty()) {
        hipEvent_t e = free_ev_.back();
        free_ev_.pop_back();
        return e;
      }
    }
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }

  void progress_loop() {
    try {
      HIP_CHECK(hipSetDevice(device_));
      for (;;) {
        std::pair<int64_t, hipEvent_t> job;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return stop_ || !pending_.empty(); });
          if (pending_.empty()) return;  // stop requested and drained
          job = pending_.front();
          pending_.pop_front();
        }
        HIP_CHECK(hipEventSynchronize(job.second));
        grp_.publish(ShmGroup::kDone, job.first + 1);
        std::lock_guard<std::mutex> g(mu_);
        free_ev_.push_back(job.second);
      }
    } catch (const std::exception& e) {
      grp_.abort(std::string("copy completion: ") + e.what());
      std::lock_guard<std::mutex> g(mu_);
      progress_error_ = e.what();
    }
  }

  int rank_, world_, device_;
  ShmGroup grp_;
  int64_t seq_ = 0;
  int64_t bytes_pulled_ = 0;
  struct Exported {
    size_t size;
    int id;
    uint64_t epoch;  // alloc_epoch() at export: a later free of the base invalidates the entry
  };
  std::map<uintptr_t, Exported> exported_;  // by base
  std::map<std::pair<int, int>, std::pair<void*, int64_t>> mapped_;  // (peer, id) -> (mapping, size)
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<int64_t, hipEvent_t>> pending_;
  std::vector<hipEvent_t> free_ev_;
  bool stop_ = false;
  struct DescSlot {
    PinnedBuffer host;
    DeviceBuffer dev;
    hipEvent_t uploaded = nullptr;
    bool used = false;
  };
  std::vector<DescSlot> descs_;
  int next_desc_ = 0;
  hipEvent_t ready_ev_ = nullptr;
  std::string progress_error_;
  std::thread progress_;
};
}  // namespace

void Exchange::wait(hipStream_t s) { HIP_CHECK(hipStreamSynchronize(s)); }

std::string exchange_probe(Exchange& ex, int device, const std::vector<std::vector<int64_t>>& send_sizes,
                           const std::vector<std::vector<int64_t>>& recv_sizes, bool host_source, int rounds,
                           int64_t export_bytes) {
  const int W = ex.world(), me = ex.rank();
  auto pattern = [](int from, int to, size_t i, int round) { return (uint8_t)((from * 31 + to * 7 + i * 3 + round) & 0xFF); };
  try {
    HIP_CHECK(hipSetDevice(device));
    if ((int)send_sizes.size() != W || (int)recv_sizes.size() != W) throw std::runtime_error("probe: bad plan");
    int64_t sb = 0, rb = 0;
    for (auto& v : send_sizes)
      for (int64_t b : v) sb += b;
    for (auto& v : recv_sizes)
      for (int64_t b : v) rb += b;
    DeviceBuffer dsend, drecv((size_t)std::max<int64_t>(rb, 16));
    PinnedBuffer hsend;
    uint8_t* sbase;
    // export_bytes > the slices: one allocation of that size (a map-output store is one multi-GB
    // export) with the slices spread over it, the last ending at its end, so peers map and read
    // beyond 4 GiB of it as the shuffle rounds will
    const int64_t alloc_bytes = std::max<int64_t>(std::max<int64_t>(sb, 16), host_source ? 0 : export_bytes);
    int64_t nslices = 0;
    for (auto& v : send_sizes) nslices += (int64_t)v.size();
    const int64_t gap = nslices > 0 ? ((alloc_bytes - sb) / nslices) & ~(int64_t)255 : 0;
    if (host_source) {
      hsend.alloc((size_t)std::max<int64_t>(sb, 16));
      sbase = hsend.as<uint8_t>();
    } else {
      dsend.alloc((size_t)alloc_bytes);
      sbase = dsend.as<uint8_t>();
    }
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct StreamGuard {
      hipStream_t s;
      ~StreamGuard() { (void)hipStreamDestroy(s); }
    } sg{st};
    for (int round = 0; round < rounds; ++round) {
      if (round >= 2) ex.wait_sent(round - 2);  // send buffer reused every round: wait for the readers
      if (round >= 1) ex.wait_sent(round - 1);
      std::vector<std::vector<Span>> send(W), recv(W);
      int64_t off = 0;
      for (int p = 0; p < W; ++p)
        for (size_t i = 0; i < send_sizes[p].size(); ++i) {
          off += gap;
          HIP_CHECK(hipMemsetAsync(sbase + off, pattern(me, p, i, round), (size_t)send_sizes[p][i], st));
          send[p].push_back(Span{sbase + off, send_sizes[p][i]});
          off += send_sizes[p][i];
        }
      off = 0;
      for (int p = 0; p < W; ++p)
        for (size_t i = 0; i < recv_sizes[p].size(); ++i) {
          recv[p].push_back(Span{drecv.as<uint8_t>() + off, recv_sizes[p][i]});
          off += recv_sizes[p][i];
        }
      HIP_CHECK(hipStreamSynchronize(st));
      ex.exchange(send, recv, st);
      ex.wait(st);
      std::vector<uint8_t> h((size_t)rb);
      if (rb) HIP_CHECK(hipMemcpy(h.data(), drecv.as(), (size_t)rb, hipMemcpyDeviceToHost));
      off = 0;
      for (int p = 0; p < W; ++p)
        for (size_t i = 0; i < recv_sizes[p].size(); ++i) {
          for (int64_t b = 0; b < recv_sizes[p][i]; ++b)
            if (h[(size_t)(off + b)] != pattern(p, me, i, round))
              throw std::runtime_error("probe: wrong bytes in slice " + std::to_string(i) + " from rank " +
                                       std::to_string(p));
          off += recv_sizes[p][i];
        }
    }
    ex.quiesce();
    return "";
  } catch (const std::exception& e) {
    return e.what();
  }
}

std::unique_ptr<Exchange> make_rccl_exchange(int rank, int world, const std::string& uid) {
  return std::make_unique<RcclExchange>(rank, world, uid);
}
std::unique_ptr<Exchange> make_local_exchange(const std::string& group, int rank, int world) {
  return std::make_unique<LocalExchange>(group, rank, world);
}
std::unique_ptr<Exchange> make_ipc_exchange(const std::string& name, int rank, int world, int device) {
  return std::make_unique<IpcExchange>(name, rank, world, device);
}

}  // namespace gpu
}  // namespace uda
