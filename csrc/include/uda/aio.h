// Asynchronous file I/O for the provider's MOF reads and the consumer's spill tier.
//
// Parity: AIOHandler (libaio, src/include/AIOHandler.h:39-105, src/CommUtils/AIOHandler.cc) with
// 4 KiB O_DIRECT alignment (AIO_ALIGNMENT) and a completion thread, and the per-disk blocking
// reader pool of src/AsyncIO/* (mapred.uda.provider.blocked.threads.per.disk). libaio/liburing are
// not available here, so the primary backend drives io_uring through raw syscalls
// (<linux/io_uring.h>); when io_uring is unavailable (old kernel, seccomp) the same interface is
// served by a pread/pwrite thread pool.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

namespace uda {

constexpr int64_t kAioAlignment = 4096;

using IoDone = std::function<void(int64_t result)>;  // bytes transferred or -errno

class AsyncIO {
 public:
  struct Options {
    int threads = 4;          // completion/worker threads
    int queue_depth = 128;    // io_uring entries
    bool prefer_uring = true;
  };
  static std::unique_ptr<AsyncIO> create(const Options& o);
  virtual ~AsyncIO() = default;
  virtual void read(int fd, int64_t off, int64_t len, void* dst, IoDone cb) = 0;
  virtual void write(int fd, int64_t off, int64_t len, const void* src, IoDone cb) = 0;
  // Block until every submitted operation completed.
  virtual void drain() = 0;
  virtual const char* backend() const = 0;
  virtual int64_t inflight() const = 0;
};

// Aligned allocation helpers for O_DIRECT buffers.
void* aligned_alloc_io(size_t bytes);
void aligned_free_io(void* p);
bool is_aligned_io(int64_t off, int64_t len, const void* p);

}  // namespace uda
