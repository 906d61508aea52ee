// AsyncIO backends: io_uring via raw syscalls, and a pread/pwrite thread pool fallback.
#include "uda/aio.h"
#include "uda/fault.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "uda/log.h"
#include "uda/thread_name.h"

namespace uda {

void* aligned_alloc_io(size_t bytes) {
  void* p = nullptr;
  size_t n = (bytes + kAioAlignment - 1) / kAioAlignment * kAioAlignment;
  if (posix_memalign(&p, (size_t)kAioAlignment, n ? n : (size_t)kAioAlignment) != 0) return nullptr;
  return p;
}
void aligned_free_io(void* p) { free(p); }
bool is_aligned_io(int64_t off, int64_t len, const void* p) {
  return off % kAioAlignment == 0 && len % kAioAlignment == 0 && ((uintptr_t)p % kAioAlignment) == 0;
}

namespace {

struct Op {
  bool is_write;
  int fd;
  int64_t off, len, done;
  uint8_t* buf;
  IoDone cb;
};

// ------------------------------------------------------------------------------- thread pool
class PoolIO : public AsyncIO {
 public:
  explicit PoolIO(int threads) {
    for (int i = 0; i < (threads > 0 ? threads : 1); ++i) thr_.emplace_back([this] { name_thread("uda-aio"); loop(); });
  }
  ~PoolIO() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : thr_) t.join();
  }
  void read(int fd, int64_t off, int64_t len, void* dst, IoDone cb) override {
    push(Op{false, fd, off, len, 0, (uint8_t*)dst, std::move(cb)});
  }
  void write(int fd, int64_t off, int64_t len, const void* src, IoDone cb) override {
    push(Op{true, fd, off, len, 0, (uint8_t*)src, std::move(cb)});
  }
  void drain() override {
    std::unique_lock<std::mutex> lk(mu_);
    idle_.wait(lk, [&] { return q_.empty() && inflight_ == 0; });
  }
  const char* backend() const override { return "threadpool"; }
  int64_t inflight() const override { return inflight_.load(); }

 private:
  void push(Op op) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(op));
      ++inflight_;
    }
    cv_.notify_one();
  }
  void loop() {
    for (;;) {
      Op op;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        op = std::move(q_.front());
        q_.pop_front();
      }
      int64_t total = 0, r = 0;
      while (total < op.len) {
        r = op.is_write ? ::pwrite(op.fd, op.buf + total, (size_t)(op.len - total), op.off + total)
                        : ::pread(op.fd, op.buf + total, (size_t)(op.len - total), op.off + total);
        if (r < 0 && errno == EINTR) continue;  // AIOHandler.cc:173-177 retries EINTR
        if (r <= 0) break;
        total += r;
      }
      int64_t res = (r < 0) ? -(int64_t)errno : total;
      if (op.cb) op.cb(res);
      {
        std::lock_guard<std::mutex> g(mu_);
        --inflight_;
      }
      idle_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<Op> q_;
  std::vector<std::thread> thr_;
  std::atomic<int64_t> inflight_{0};
  bool stop_ = false;
};

// ------------------------------------------------------------------------------- io_uring
int sys_setup(unsigned entries, io_uring_params* p) { return (int)syscall(__NR_io_uring_setup, entries, p); }
int sys_enter(int fd, unsigned to_submit, unsigned min_complete, unsigned flags) {
  return (int)syscall(__NR_io_uring_enter, fd, to_submit, min_complete, flags, nullptr, 0);
}

class UringIO : public AsyncIO {
 public:
  static std::unique_ptr<UringIO> try_create(int depth) {
    std::unique_ptr<UringIO> u(new UringIO());
    if (!u->init(depth)) return nullptr;
    return u;
  }
  ~UringIO() override {
    if (reaper_.joinable()) {
      drain();
      {
        std::lock_guard<std::mutex> g(sq_mu_);
        stop_ = true;
      }
      submit_op(nullptr);  // wake the reaper with a NOP
      reaper_.join();
    }
    if (sq_ptr_) munmap(sq_ptr_, sq_sz_);
    if (cq_ptr_ && cq_ptr_ != sq_ptr_) munmap(cq_ptr_, cq_sz_);
    if (sqes_) munmap(sqes_, sqes_sz_);
    if (ring_fd_ >= 0) close(ring_fd_);
  }
  void read(int fd, int64_t off, int64_t len, void* dst, IoDone cb) override {
    submit_op(new Op{false, fd, off, len, 0, (uint8_t*)dst, std::move(cb)});
  }
  void write(int fd, int64_t off, int64_t len, const void* src, IoDone cb) override {
    submit_op(new Op{true, fd, off, len, 0, (uint8_t*)src, std::move(cb)});
  }
  void drain() override {
    std::unique_lock<std::mutex> lk(idle_mu_);
    idle_.wait(lk, [&] { return inflight_.load() == 0; });
  }
  const char* backend() const override { return "io_uring"; }
  int64_t inflight() const override { return inflight_.load(); }

 private:
  UringIO() = default;
  bool init(int depth) {
    io_uring_params p;
    std::memset(&p, 0, sizeof(p));
    ring_fd_ = sys_setup((unsigned)depth, &p);
    if (ring_fd_ < 0) return false;
    entries_ = p.sq_entries;
    sq_sz_ = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    cq_sz_ = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    const bool single = p.features & IORING_FEAT_SINGLE_MMAP;
    if (single) sq_sz_ = cq_sz_ = std::max(sq_sz_, cq_sz_);
    sq_ptr_ = mmap(nullptr, sq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd_, IORING_OFF_SQ_RING);
    if (sq_ptr_ == MAP_FAILED) return false;
    cq_ptr_ = single ? sq_ptr_
                     : mmap(nullptr, cq_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd_,
                            IORING_OFF_CQ_RING);
    if (cq_ptr_ == MAP_FAILED) return false;
    sqes_sz_ = p.sq_entries * sizeof(io_uring_sqe);
    sqes_ = (io_uring_sqe*)mmap(nullptr, sqes_sz_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd_,
                                IORING_OFF_SQES);
    if (sqes_ == MAP_FAILED) return false;
    auto* sq = (uint8_t*)sq_ptr_;
    sq_head_ = (unsigned*)(sq + p.sq_off.head);
    sq_tail_ = (unsigned*)(sq + p.sq_off.tail);
    sq_mask_ = (unsigned*)(sq + p.sq_off.ring_mask);
    sq_array_ = (unsigned*)(sq + p.sq_off.array);
    auto* cq = (uint8_t*)cq_ptr_;
    cq_head_ = (unsigned*)(cq + p.cq_off.head);
    cq_tail_ = (unsigned*)(cq + p.cq_off.tail);
    cq_mask_ = (unsigned*)(cq + p.cq_off.ring_mask);
    cqes_ = (io_uring_cqe*)(cq + p.cq_off.cqes);
    // probe: a NOP must complete, otherwise fall back (seccomp/emulation can stub io_uring)
    reaper_ = std::thread([this] { reap(); });
    struct Probe {
      std::mutex m;
      std::condition_variable c;
      bool fired = false, ok = false;
    };
    auto probe = std::make_shared<Probe>();
    Op* nop = new Op{false, -1, 0, 0, 0, nullptr, [probe](int64_t r) {
                       std::lock_guard<std::mutex> g(probe->m);
                       probe->ok = (r == 0);
                       probe->fired = true;
                       probe->c.notify_all();
                     }};
    submit_op(nop, /*is_nop=*/true);
    std::unique_lock<std::mutex> lk(probe->m);
    probe->c.wait_for(lk, std::chrono::seconds(2), [&] { return probe->fired; });
    if (!probe->fired || !probe->ok) {
      UDA_LOG(kWarn, "io_uring probe failed; using thread pool");
      return false;  // destructor cleans up (the reaper exits on stop_)
    }
    return true;
  }

  void submit_op(Op* op, bool is_nop = false) {
    std::unique_lock<std::mutex> lk(sq_mu_);
    // bound in-flight ops to the ring size
    space_.wait(lk, [&] { return inflight_sq_ < (int64_t)entries_; });
    const unsigned tail = *sq_tail_;
    const unsigned idx = tail & *sq_mask_;
    io_uring_sqe* e = &sqes_[idx];
    std::memset(e, 0, sizeof(*e));
    if (!op || is_nop) {
      e->opcode = IORING_OP_NOP;
    } else {
      e->opcode = op->is_write ? IORING_OP_WRITE : IORING_OP_READ;
      e->fd = op->fd;
      e->off = (uint64_t)(op->off + op->done);
      e->addr = (uint64_t)(uintptr_t)(op->buf + op->done);
      e->len = (unsigned)std::min<int64_t>(op->len - op->done, 1 << 30);
    }
    e->user_data = (uint64_t)(uintptr_t)op;
    sq_array_[idx] = idx;
    __atomic_store_n(sq_tail_, tail + 1, __ATOMIC_RELEASE);
    ++inflight_sq_;
    if (op && !is_nop) ++inflight_;
    int r;
    do {
      r = sys_enter(ring_fd_, 1, 0, 0);
    } while (r < 0 && errno == EINTR);
  }

  void reap() {
    for (;;) {
      int r = sys_enter(ring_fd_, 0, 1, IORING_ENTER_GETEVENTS);
      if (r < 0 && errno != EINTR && errno != EAGAIN && errno != EBUSY) {
        UDA_LOG(kError, "io_uring_enter failed: %s", strerror(errno));
        return;
      }
      unsigned head = *cq_head_;
      const unsigned tail = __atomic_load_n(cq_tail_, __ATOMIC_ACQUIRE);
      bool any = false;
      while (head != tail) {
        io_uring_cqe* c = &cqes_[head & *cq_mask_];
        Op* op = (Op*)(uintptr_t)c->user_data;
        const int res = c->res;
        ++head;
        any = true;
        {
          std::lock_guard<std::mutex> g(sq_mu_);
          --inflight_sq_;
        }
        space_.notify_all();
        if (!op) continue;  // wake-up NOP
        if (op->fd < 0) {   // probe NOP
          op->cb(res);
          delete op;
          continue;
        }
        if (res > 0 && op->done + res < op->len) {  // short transfer: resubmit the rest
          op->done += res;
          __atomic_store_n(cq_head_, head, __ATOMIC_RELEASE);
          submit_op(op);
          --inflight_;  // submit_op counted it again
          continue;
        }
        const int64_t result = (res < 0) ? res : op->done + res;
        if (op->cb) op->cb(result);
        delete op;
        {
          std::lock_guard<std::mutex> g(idle_mu_);
          --inflight_;
        }
        idle_.notify_all();
      }
      __atomic_store_n(cq_head_, head, __ATOMIC_RELEASE);
      {
        std::lock_guard<std::mutex> g(sq_mu_);
        if (stop_ && inflight_sq_ == 0 && !any) return;
        if (stop_ && inflight_sq_ == 0) return;
      }
    }
  }

  int ring_fd_ = -1;
  unsigned entries_ = 0;
  void* sq_ptr_ = nullptr;
  void* cq_ptr_ = nullptr;
  size_t sq_sz_ = 0, cq_sz_ = 0, sqes_sz_ = 0;
  io_uring_sqe* sqes_ = nullptr;
  unsigned *sq_head_ = nullptr, *sq_tail_ = nullptr, *sq_mask_ = nullptr, *sq_array_ = nullptr;
  unsigned *cq_head_ = nullptr, *cq_tail_ = nullptr, *cq_mask_ = nullptr;
  io_uring_cqe* cqes_ = nullptr;
  std::mutex sq_mu_, idle_mu_;
  std::condition_variable space_, idle_;
  int64_t inflight_sq_ = 0;
  std::atomic<int64_t> inflight_{0};
  bool stop_ = false;
  std::thread reaper_;
};

}  // namespace

namespace {
// Fault-injection decorator (UDA_FAULT_AIO=<n>: the n-th operation completes with -EIO).
class FaultIO : public AsyncIO {
 public:
  explicit FaultIO(std::unique_ptr<AsyncIO> in) : in_(std::move(in)) {}
  void read(int fd, int64_t off, int64_t len, void* dst, IoDone cb) override {
    if (fault_hit("AIO")) return cb(-EIO);
    in_->read(fd, off, len, dst, std::move(cb));
  }
  void write(int fd, int64_t off, int64_t len, const void* src, IoDone cb) override {
    if (fault_hit("AIO")) return cb(-EIO);
    in_->write(fd, off, len, src, std::move(cb));
  }
  void drain() override { in_->drain(); }
  const char* backend() const override { return in_->backend(); }
  int64_t inflight() const override { return in_->inflight(); }

 private:
  std::unique_ptr<AsyncIO> in_;
};
}  // namespace

std::unique_ptr<AsyncIO> AsyncIO::create(const Options& o) {
  const char* env = std::getenv("UDA_AIO_BACKEND");
  bool uring = o.prefer_uring && !(env && std::string(env) == "threadpool");
  std::unique_ptr<AsyncIO> io;
  if (uring) io = UringIO::try_create(o.queue_depth);
  if (!io) io = std::make_unique<PoolIO>(o.threads);
  return std::make_unique<FaultIO>(std::move(io));
}

}  // namespace uda
