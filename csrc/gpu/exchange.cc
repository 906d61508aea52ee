#include "exchange.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <map>
#include <mutex>
#include <stdexcept>

#include "device_engine.h"

namespace uda {
namespace gpu {

namespace {
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r) + " in " + what);
}
#define NCCL_CHECK(x) nccl_check((x), #x)

// ------------------------------------------------------------------------------------ RCCL
class RcclExchange : public Exchange {
 public:
  RcclExchange(int rank, int world, const std::string& uid) : rank_(rank), world_(world) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
    HIP_CHECK(hipMalloc(&d_counts_, 1));
    if (const char* t = std::getenv("UDA_RCCL_TIMEOUT_S")) timeout_ = std::chrono::seconds(std::max(1, std::atoi(t)));
  }
  ~RcclExchange() override {
    if (comm_) (aborted_ ? ncclCommAbort(comm_) : ncclCommDestroy(comm_));
    if (d_counts_) (void)hipFree(d_counts_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "rccl"; }

  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t s) override {
    const size_t bytes = n * (size_t)world_ * 8;
    if (bytes * 2 > counts_cap_) {
      if (d_counts_) HIP_CHECK(hipFree(d_counts_));
      HIP_CHECK(hipMalloc(&d_counts_, bytes * 2));
      counts_cap_ = bytes * 2;
    }
    int64_t* ds = (int64_t*)d_counts_;
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

  void alltoallv(const uint8_t* send, const int64_t* sb, const int64_t* sd, uint8_t* recv, const int64_t* rb,
                 const int64_t* rd, hipStream_t s) override {
    NCCL_CHECK(ncclGroupStart());
    for (int k = 1; k < world_; ++k) {
      const int to = (rank_ + k) % world_;      // rotating order spreads the xGMI link load
      const int from = (rank_ - k + world_) % world_;
      if (sb[to] > 0) NCCL_CHECK(ncclSend(send + sd[to], (size_t)sb[to], ncclUint8, to, comm_, s));
      if (rb[from] > 0) NCCL_CHECK(ncclRecv(recv + rd[from], (size_t)rb[from], ncclUint8, from, comm_, s));
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
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
  bool aborted_ = false;
  std::chrono::seconds timeout_{900};
  void* d_counts_ = nullptr;
  size_t counts_cap_ = 0;
};

// ------------------------------------------------------------------------------------ local group
struct Group {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  struct Post {
    const void* send = nullptr;
    const int64_t* sb = nullptr;
    const int64_t* sd = nullptr;
    hipEvent_t ready = nullptr;  // sender's data is packed
    hipEvent_t done = nullptr;   // this rank finished reading its peers' data
  };
  std::vector<Post> posts;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};

std::mutex g_groups_mu;
std::map<std::string, std::shared_ptr<Group>> g_groups;

class LocalExchange : public Exchange {
 public:
  LocalExchange(const std::string& name, int rank, int world) : rank_(rank), world_(world) {
    std::lock_guard<std::mutex> g(g_groups_mu);
    auto& grp = g_groups[name];
    if (!grp) {
      grp = std::make_shared<Group>();
      grp->world = world;
      grp->posts.resize(world);
    }
    if (grp->world != world) throw std::runtime_error("local exchange: world mismatch");
    group_ = grp;
    HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  ~LocalExchange() override {
    (void)hipEventDestroy(ready_);
    (void)hipEventDestroy(done_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  const char* name() const override { return "local"; }

  void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t) override {
    Group& g = *group_;
    g.posts[rank_].send = send;
    g.barrier();
    for (int p = 0; p < world_; ++p)
      std::memcpy(recv + p * n, (const int64_t*)g.posts[p].send + (size_t)rank_ * n, n * 8);
    g.barrier();
  }

  void alltoallv(const uint8_t* send, const int64_t* sb, const int64_t* sd, uint8_t* recv, const int64_t* rb,
                 const int64_t* rd, hipStream_t s) override {
    Group& g = *group_;
    HIP_CHECK(hipEventRecord(ready_, s));
    g.posts[rank_].send = send;
    g.posts[rank_].sb = sb;
    g.posts[rank_].sd = sd;
    g.posts[rank_].ready = ready_;
    g.posts[rank_].done = done_;
    g.barrier();
    for (int k = 1; k < world_; ++k) {
      const int from = (rank_ - k + world_) % world_;
      const auto& p = g.posts[from];
      if (p.sb[rank_] != rb[from])
        throw std::runtime_error("local exchange: size mismatch between sender and receiver plans");
      if (rb[from] <= 0) continue;
      HIP_CHECK(hipStreamWaitEvent(s, p.ready, 0));
      HIP_CHECK(hipMemcpyAsync(recv + rd[from], (const uint8_t*)p.send + p.sd[rank_], (size_t)rb[from],
                               hipMemcpyDeviceToDevice, s));
    }
    HIP_CHECK(hipEventRecord(done_, s));
    g.barrier();
    // send completion: my packed buffer may be reused only after every receiver copied it
    for (int p = 0; p < world_; ++p)
      if (p != rank_) HIP_CHECK(hipStreamWaitEvent(s, g.posts[p].done, 0));
    g.barrier();  // posts (and events) stay valid until everyone enqueued its waits
  }

 private:
  int rank_, world_;
  std::shared_ptr<Group> group_;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
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
