#include "exchange.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "device_engine.h"

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
  const char* name() const override { return pack_ ? "rccl-packed" : "rccl"; }

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
  std::vector<const std::vector<std::vector<Span>>*> sends;  // per rank, valid between barriers
  std::vector<const int64_t*> counts;
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
    }
    if (grp->world != world) throw std::runtime_error("local exchange: world mismatch");
    group_ = grp;
  }
  ~LocalExchange() override {
    std::lock_guard<std::mutex> g(g_groups_mu);
    auto it = g_groups.find(name_);
    if (it != g_groups.end() && it->second == group_ && group_.use_count() <= 2) g_groups.erase(it);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "local"; }

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
    g.sends[rank_] = &send;
    g.barrier();
    try {
      for (int k = 1; k < world_; ++k) {
        const int from = (rank_ - k + world_) % world_;
        const auto& theirs = (*g.sends[from])[rank_];
        const auto& mine = recv[from];
        if (theirs.size() != mine.size())
          throw std::runtime_error("local exchange: slice count mismatch between sender and receiver plans");
        for (size_t i = 0; i < mine.size(); ++i) {
          if (theirs[i].bytes != mine[i].bytes)
            throw std::runtime_error("local exchange: slice size mismatch between sender and receiver plans");
          HIP_CHECK(hipMemcpyAsync(const_cast<uint8_t*>(mine[i].ptr), theirs[i].ptr, (size_t)mine[i].bytes,
                                   hipMemcpyDefault, s));
        }
      }
    } catch (...) {
      g.abort();
      throw;
    }
    g.barrier();  // peers' send lists are no longer read
  }

 private:
  std::string name_;
  int rank_, world_;
  std::shared_ptr<Group> group_;
};
}  // namespace

void Exchange::wait(hipStream_t s) { HIP_CHECK(hipStreamSynchronize(s)); }

std::unique_ptr<Exchange> make_rccl_exchange(int rank, int world, const std::string& uid) {
  return std::make_unique<RcclExchange>(rank, world, uid);
}
std::unique_ptr<Exchange> make_local_exchange(const std::string& group, int rank, int world) {
  return std::make_unique<LocalExchange>(group, rank, world);
}

}  // namespace gpu
}  // namespace uda
