// Disk tier of the partition store. See disk_store.h.
#include "disk_store.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <stdexcept>

#include "device_engine.h"
#include "sdma.h"
#include "uda/log.h"

namespace uda {
namespace gpu {

namespace {
int64_t align_dn(int64_t v) { return v / kAioAlignment * kAioAlignment; }
int64_t align_upio(int64_t v) { return (v + kAioAlignment - 1) / kAioAlignment * kAioAlignment; }
}  // namespace

DiskStore::DiskStore(int device, const std::vector<std::string>& dirs, const std::string& tag, int nfiles,
                     int chunks, int64_t chunk_bytes)
    : nchunks_(std::max(2, chunks)), chunk_(align_upio(std::max<int64_t>(chunk_bytes, 1 << 20))) {
  std::vector<std::string> d = dirs.empty() ? std::vector<std::string>{"/tmp"} : dirs;
  for (int f = 0; f < nfiles; ++f) {
    const std::string p = d[(size_t)f % d.size()] + "/uda.store." + tag + "." + std::to_string(f);
    int fd = ::open(p.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC | O_DIRECT, 0600);
    if (fd < 0 && errno == EINVAL) {  // file system without O_DIRECT
      direct_ = false;
      fd = ::open(p.c_str(), O_CREAT | O_TRUNC | O_RDWR | O_CLOEXEC, 0600);
    }
    if (fd < 0) throw std::runtime_error("disk store: cannot create " + p + ": " + strerror(errno));
    paths_.push_back(p);
    fds_.push_back(fd);
  }
  sizes_.assign(nfiles, 0);
  AsyncIO::Options o;
  o.threads = 4;
  o.queue_depth = 64;
  aio_ = AsyncIO::create(o);
  ring_ = static_cast<uint8_t*>(hip_host_alloc_on_node((size_t)(nchunks_ * chunk_), device_numa_node(device)));
  ev_.resize(nchunks_);
  for (auto& e : ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  pending_.assign(nchunks_, false);
}

DiskStore::~DiskStore() {
  if (aio_) aio_->drain();
  for (size_t i = 0; i < ev_.size(); ++i) {
    if (pending_[i]) (void)hipEventSynchronize(ev_[i]);
    (void)hipEventDestroy(ev_[i]);
  }
  if (ring_) pinned_host_free(ring_);
  for (size_t f = 0; f < fds_.size(); ++f) {
    if (fds_[f] >= 0) ::close(fds_[f]);
    ::unlink(paths_[f].c_str());
  }
}

std::string DiskStore::describe() const {
  return std::string("disk[") + (paths_.empty() ? "" : paths_[0].substr(0, paths_[0].rfind('/'))) + " files=" +
         std::to_string(paths_.size()) + " io=" + aio_->backend() + (direct_ ? " O_DIRECT" : " buffered") + "]";
}

void DiskStore::write_file(int f, const uint8_t* src_dev, int64_t len, hipStream_t s) {
  const int64_t padded = align_upio(len);
  int64_t err = 0;
  for (int64_t off = 0; off < padded; off += chunk_ * nchunks_) {
    // D2H a window of chunks, then write them out (the ring is free again when the writes drained)
    const int64_t win = std::min(chunk_ * nchunks_, padded - off);
    const int64_t have = std::max<int64_t>(0, std::min(win, len - off));
    if (have > 0) HIP_CHECK(hipMemcpyAsync(ring_, src_dev + off, (size_t)have, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (have < win) std::memset(ring_ + have, 0, (size_t)(win - have));
    for (int64_t o = 0; o < win; o += chunk_) {
      const int64_t n = std::min(chunk_, win - o);
      aio_->write(fds_[f], off + o, n, ring_ + o, [&err, n](int64_t r) {
        if (r != n) err = r < 0 ? r : -EIO;
      });
    }
    aio_->drain();
    if (err) throw std::runtime_error("disk store: write failed on " + paths_[f] + ": " + strerror((int)-err));
  }
  sizes_[f] = padded;
  bytes_written_ += padded;
}

void DiskStore::stage(const std::vector<Piece>& pieces, hipStream_t s) {
  struct Sub {
    int file;
    int64_t off, len;
    uint8_t* dst;
  };
  std::vector<Sub> subs;
  const int64_t span = chunk_ - kAioAlignment;  // an aligned superset of a sub-piece fits one chunk
  for (const Piece& p : pieces)
    for (int64_t o = 0; o < p.len; o += span) subs.push_back(Sub{p.file, p.off + o, std::min(span, p.len - o), p.dst + o});
  const int64_t n = (int64_t)subs.size();
  std::vector<int64_t> result((size_t)n, 0);
  std::vector<char> done((size_t)n, 0);
  std::vector<int64_t> a0((size_t)n, 0);
  int64_t next_submit = 0, next_finish = 0;
  while (next_finish < n) {
    while (next_submit < n && next_submit - next_finish < nchunks_) {
      const int slot = (int)(next_submit % nchunks_);
      if (pending_[slot]) {  // the chunk's previous H2D must have read it
        HIP_CHECK(hipEventSynchronize(ev_[slot]));
        pending_[slot] = false;
      }
      const Sub& sb = subs[(size_t)next_submit];
      const int64_t lo = direct_ ? align_dn(sb.off) : sb.off;
      int64_t hi = direct_ ? align_upio(sb.off + sb.len) : sb.off + sb.len;
      hi = std::min(hi, std::max(sizes_[(size_t)sb.file], sb.off + sb.len));
      a0[(size_t)next_submit] = lo;
      const int64_t i = next_submit;
      aio_->read(fds_[(size_t)sb.file], lo, hi - lo, ring_ + (int64_t)slot * chunk_, [this, i, &result, &done](int64_t r) {
        std::lock_guard<std::mutex> g(mu_);
        result[(size_t)i] = r;
        done[(size_t)i] = 1;
        cv_.notify_all();
      });
      ++next_submit;
    }
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return done[(size_t)next_finish] != 0; });
    }
    const Sub& sb = subs[(size_t)next_finish];
    const int64_t need = sb.off + sb.len - a0[(size_t)next_finish];
    if (result[(size_t)next_finish] < need) {
      aio_->drain();
      throw std::runtime_error("disk store: short read from " + paths_[(size_t)sb.file]);
    }
    const int slot = (int)(next_finish % nchunks_);
    HIP_CHECK(hipMemcpyAsync(sb.dst, ring_ + (int64_t)slot * chunk_ + (sb.off - a0[(size_t)next_finish]), (size_t)sb.len,
                             hipMemcpyHostToDevice, s));
    HIP_CHECK(hipEventRecord(ev_[slot], s));
    pending_[slot] = true;
    bytes_read_ += sb.len;
    ++next_finish;
  }
}

std::vector<uint8_t> DiskStore::read_host(int f, int64_t off, int64_t len) {
  std::vector<uint8_t> out((size_t)len);
  const int64_t lo = align_dn(off), hi = align_upio(off + len);
  void* b = aligned_alloc_io((size_t)(hi - lo));
  const ssize_t r = ::pread(fds_[(size_t)f], b, (size_t)(hi - lo), lo);
  if (r < off + len - lo) {
    aligned_free_io(b);
    throw std::runtime_error("disk store: short read from " + paths_[(size_t)f]);
  }
  std::memcpy(out.data(), static_cast<uint8_t*>(b) + (off - lo), (size_t)len);
  aligned_free_io(b);
  return out;
}

}  // namespace gpu
}  // namespace uda
