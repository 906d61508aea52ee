#include "supplier.h"

#include <fcntl.h>
#include <unistd.h>

#include <cstring>

#include "../gpu/device_ptr.h"
#include "uda/log.h"
#include "uda/trace.h"
#include "uda/thread_name.h"

namespace uda {

Supplier::Supplier(const NetlevOptions& net, const Options& o, Host* host) : net_(net), opt_(o), host_(host) {
  AsyncIO::Options ao;
  ao.threads = o.io_threads;
  aio_ = AsyncIO::create(ao);
}

Supplier::~Supplier() { stop(); }

void Supplier::start() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = false;
  }
  for (int i = 0; i < std::max(1, opt_.workers); ++i) workers_.emplace_back([this] { name_thread("uda-supply"); worker(); });
  if (opt_.transport == "tcp")
    server_ = make_tcp_server(net_.data_port, net_.wqes_per_conn, opt_.bind_addr);
  else
    server_ = make_loopback_server(opt_.loopback_host);
  server_->start(this);
  UDA_LOG(kInfo, "MOFSupplier started: transport=%s port=%d io=%s", opt_.transport.c_str(), port(),
          aio_->backend());
}

void Supplier::stop() {
  if (server_) server_->stop();
  server_.reset();
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
  workers_.clear();
  if (aio_) aio_->drain();
  set_store(nullptr);  // after the workers: no fetch is being answered from it
  std::lock_guard<std::mutex> g(fd_mu_);
  for (auto& kv : fds_)
    if (kv.second.fd >= 0) ::close(kv.second.fd);
  fds_.clear();
}

void Supplier::register_mof(const std::string& job, const std::string& map, const uint8_t* data, int64_t len,
                            std::vector<IndexRec> index, int device) {
  MemMof m{data, len, std::move(index)};
  m.device = device;
  if (device >= 0) {
    const gpu::IpcExport ex = gpu::ipc_export(data);
    m.ipc_handle = ex.handle_hex;
    m.ipc_base = ex.base;
  }
  std::lock_guard<std::mutex> g(idx_mu_);
  mem_[job + "|" + map] = std::move(m);
}

void Supplier::job_over(const std::string& job) {
  if (auto st = store()) st->job_over(job);
  std::lock_guard<std::mutex> g(idx_mu_);
  const std::string pre = job + "|";
  for (auto it = idx_cache_.begin(); it != idx_cache_.end();)
    it = it->first.compare(0, pre.size(), pre) == 0 ? idx_cache_.erase(it) : std::next(it);
}

std::string Supplier::hbm_stats_json() {
  auto st = store();
  return st ? st->stats_json() : "{}";
}

void Supplier::serve(const FetchRequest& req, uint8_t* dst, FetchDone done) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!stop_) {
      q_.push_back(Job{req, dst, std::move(done)});
      cv_.notify_one();
      return;
    }
  }
  FetchAck a;  // stopped: no worker will take the request, complete it now
  a.status = -11;
  a.error = "MOFSupplier stopped";
  done(a);
}

bool Supplier::serve_ref(const FetchRequest& req, RefDone done) {
  if (req.buf_len <= 0) return false;  // descriptor fetches and releases carry no bytes
  if (opt_.copy_serve) return false;  // A/B: every answer through a chunk copy
  std::lock_guard<std::mutex> g(mu_);
  if (stop_) return false;  // serve() answers it (with the stopped error)
  q_.push_back(Job{req, nullptr, nullptr, std::move(done)});
  cv_.notify_one();
  return true;
}

void Supplier::worker() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      j = std::move(q_.front());
      q_.pop_front();
    }
    try {
      if (j.ref_done)
        process_ref(j);
      else
        process(j);
    } catch (const std::exception& e) {
      FetchAck a;
      a.status = -9;
      a.error = e.what();
      if (j.ref_done)
        j.ref_done(a, Bytes{});
      else
        j.done(a);
    }
  }
}

bool Supplier::resolve(const FetchRequest& req, IndexRec* rec, const MemMof** mem) {
  *mem = nullptr;
  std::lock_guard<std::mutex> g(idx_mu_);
  auto m = mem_.find(req.job_id + "|" + req.map_id);
  if (m != mem_.end()) {
    if (req.reduce_id < 0 || req.reduce_id >= (int)m->second.index.size()) return false;
    *rec = m->second.index[req.reduce_id];
    *mem = &m->second;
    return true;
  }
  const std::string key = req.job_id + "|" + req.map_id + "|" + std::to_string(req.reduce_id);
  auto c = idx_cache_.find(key);
  if (c != idx_cache_.end()) {
    *rec = c->second;
    return true;
  }
  // first touch: ask the host (getPathUda -> IndexRecordBridge)
  IndexRec r;
  if (!host_ || !host_->get_path(req.job_id, req.map_id, req.reduce_id, &r)) return false;
  idx_cache_[key] = r;
  *rec = r;
  return true;
}

int Supplier::acquire_fd(const std::string& path) {
  std::lock_guard<std::mutex> g(fd_mu_);
  auto it = fds_.find(path);
  if (it == fds_.end()) {
    // evict idle descriptors beyond the bound
    if ((int)fds_.size() >= opt_.max_open_files) {
      for (auto e = fds_.begin(); e != fds_.end();) {
        if (e->second.refs == 0) {
          ::close(e->second.fd);
          e = fds_.erase(e);
        } else {
          ++e;
        }
      }
    }
    int flags = O_RDONLY | O_CLOEXEC | (opt_.odirect ? O_DIRECT : 0);
    int fd = ::open(path.c_str(), flags);
    if (fd < 0 && opt_.odirect) fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);  // fs without O_DIRECT
    if (fd < 0) return -1;
    it = fds_.emplace(path, OpenFile{fd, 0, 0}).first;
  }
  it->second.refs++;
  it->second.last_use = ++fd_clock_;
  return it->second.fd;
}

void Supplier::release_fd(const std::string& path) {
  std::lock_guard<std::mutex> g(fd_mu_);
  auto it = fds_.find(path);
  if (it != fds_.end() && it->second.refs > 0) it->second.refs--;
}

void Supplier::process(Job& j) {
  requests_++;
  IndexRec rec;
  const MemMof* mem = nullptr;
  FetchAck ack;
  if (j.req.buf_len == kDescriptorRelease) {
    // the reducer is done with descriptors it fetched (chunk release on SEND completion,
    // src/MOFServer/IndexInfo.cc:276-301): the store may free the MOFs nobody holds any more
    if (auto st = store()) {
      if (j.req.map_id == "*") {
        st->release_holder(j.req.job_id, j.req.holder);
      } else if (resolve(j.req, &rec, &mem) && !mem) {
        st->release(rec.path, j.req.holder);
      }
    }
    releases_++;
    j.done(ack);
    return;
  }
  if (!resolve(j.req, &rec, &mem)) {
    ack.status = -2;
    ack.error = "cannot resolve MOF " + j.req.job_id + "/" + j.req.map_id + "/" + std::to_string(j.req.reduce_id);
    j.done(ack);
    return;
  }
  if ((int)rec.path.size() > kMofPathMax) {  // MOF_PATH_SIZE_TOO_LONG (IndexInfo.cc:265-270)
    ack.status = -3;
    ack.error = "MOF path too long";
    j.done(ack);
    return;
  }
  ack.raw_len = rec.raw_length;
  ack.part_len = rec.part_length;
  ack.mof_offset = rec.start_offset;
  ack.path = rec.path;
  if (j.req.buf_len == kDescriptorFetch) {
    // zero-copy fetch: the reducer reads the partition where it lives (RDMA WRITE analogue)
    if (first_desc_boot_ms_.load() == 0) {
      timespec ts{};
      clock_gettime(CLOCK_BOOTTIME, &ts);
      double zero = 0;
      first_desc_boot_ms_.compare_exchange_strong(zero, (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6);
    }
    std::string why;
    std::shared_ptr<DeviceStore> st = mem ? nullptr : store();
    if (st) {
      // a Hadoop-written MOF file, made resident in the provider's HBM store (this process's or the node
      // daemon's): answered once the file has landed up to the end of this partition (the loader fills
      // files in turn)
      auto done = j.done;
      const bool taken = st->acquire(
          j.req.job_id, rec.path, j.req.holder, rec.start_offset, rec.part_length,
          [this, ack, done](int status, const std::string& desc) mutable {
            if (status != 0) {
              ack.status = status;  // kNotDeviceResident: the reducer fetches the bytes instead
              ack.error = desc;
            } else {
              ack.path = desc;
              ack.sent = 0;
              descriptors_++;
            }
            done(ack);
          },
          &why);
      if (taken) return;
    }
    if (!mem || mem->device < 0) {
      ack.status = kNotDeviceResident;
      ack.error = "MOF is not device-resident";
    } else if (rec.start_offset + rec.part_length > mem->len) {
      ack.status = -4;
      ack.error = "index beyond registered MOF";
    } else {
      gpu::IpcExport ex;
      ex.handle_hex = mem->ipc_handle;
      ex.base = mem->ipc_base;
      ack.path = gpu::make_device_descriptor(mem->device, mem->data + rec.start_offset, ex);
      ack.sent = 0;
      descriptors_++;
    }
    j.done(ack);
    return;
  }
  const int64_t remaining = rec.part_length - j.req.fetched;
  const int64_t len = std::max<int64_t>(0, std::min<int64_t>(remaining, j.req.buf_len));
  ack.sent = len;
  if (len == 0) {
    j.done(ack);
    return;
  }
  const int64_t off = rec.start_offset + j.req.fetched;
  if (mem) {
    if (off + len > mem->len) {
      ack.status = -4;
      ack.error = "index beyond registered MOF";
      j.done(ack);
      return;
    }
    const int64_t tc = trace::host_enabled() ? trace::now_ns() : 0;
    if (mem->device >= 0)
      gpu::copy_device_to_host(j.dst, mem->data + off, len);
    else
      std::memcpy(j.dst, mem->data + off, (size_t)len);
    if (tc) trace::host_event("serve_copy", len, (int64_t)(uintptr_t)j.dst, tc, trace::now_ns());
    bytes_ += len;
    j.done(ack);
    return;
  }
  const int fd = acquire_fd(rec.path);
  if (fd < 0) {
    ack.status = -5;
    ack.error = "cannot open " + rec.path + ": " + strerror(errno);
    j.done(ack);
    return;
  }
  const std::string path = rec.path;
  auto done = std::move(j.done);
  if (opt_.odirect) {
    // aligned read into a bounce chunk (aio_read_chunk_data alignment math, IndexInfo.cc:304-335)
    const int64_t aoff = off - off % kAioAlignment;
    const int64_t alen = ((off + len - aoff) + kAioAlignment - 1) / kAioAlignment * kAioAlignment;
    uint8_t* bounce = (uint8_t*)aligned_alloc_io((size_t)alen);
    uint8_t* dst = j.dst;
    aio_->read(fd, aoff, alen, bounce, [this, bounce, dst, off, aoff, len, ack, done, path](int64_t r) mutable {
      if (r < off - aoff + len) {
        ack.status = -6;
        ack.error = "short read";
      } else {
        std::memcpy(dst, bounce + (off - aoff), (size_t)len);
        bytes_ += len;
      }
      aligned_free_io(bounce);
      release_fd(path);
      done(ack);
    });
  } else {
    aio_->read(fd, off, len, j.dst, [this, len, ack, done, path](int64_t r) mutable {
      if (r != len) {
        ack.status = -6;
        ack.error = "short read (" + std::to_string(r) + " of " + std::to_string(len) + ")";
      } else {
        bytes_ += len;
      }
      release_fd(path);
      done(ack);
    });
  }
}

}  // namespace uda

namespace uda {

void Supplier::process_ref(Job& j) {
  requests_++;
  IndexRec rec;
  const MemMof* mem = nullptr;
  FetchAck ack;
  RefDone done = std::move(j.ref_done);
  if (!resolve(j.req, &rec, &mem)) {
    ack.status = -2;
    ack.error = "cannot resolve MOF " + j.req.job_id + "/" + j.req.map_id + "/" + std::to_string(j.req.reduce_id);
    return done(ack, Bytes{});
  }
  if ((int)rec.path.size() > kMofPathMax) {
    ack.status = -3;
    ack.error = "MOF path too long";
    return done(ack, Bytes{});
  }
  ack.raw_len = rec.raw_length;
  ack.part_len = rec.part_length;
  ack.mof_offset = rec.start_offset;
  ack.path = rec.path;
  const int64_t len = std::max<int64_t>(0, std::min<int64_t>(rec.part_length - j.req.fetched, j.req.buf_len));
  ack.sent = len;
  const int64_t off = rec.start_offset + j.req.fetched;
  if (len == 0) return done(ack, Bytes{});
  if (mem) {
    if (off + len > mem->len) {
      ack.status = -4;
      ack.error = "index beyond registered MOF";
      return done(ack, Bytes{});
    }
    Bytes b;
    if (mem->device < 0) {
      b.ptr = mem->data + off;  // the registered memory itself goes to the socket
    } else {
      uint8_t* chunk = new uint8_t[(size_t)len];
      gpu::copy_device_to_host(chunk, mem->data + off, len);
      b.ptr = chunk;
      b.release = [chunk] { delete[] chunk; };
    }
    bytes_ += len;
    return done(ack, std::move(b));
  }
  const int fd = acquire_fd(rec.path);
  if (fd < 0) {
    ack.status = -5;
    ack.error = "cannot open " + rec.path + ": " + strerror(errno);
    return done(ack, Bytes{});
  }
  const std::string path = rec.path;
  if (!opt_.odirect) {
    // a file range: the transport sends it from the page cache (sendfile), no copy through this process
    Bytes b;
    b.fd = fd;
    b.file_off = off;
    b.release = [this, path] { release_fd(path); };
    bytes_ += len;
    return done(ack, std::move(b));
  }
  // O_DIRECT: aligned read into a bounce chunk, sent from there
  const int64_t aoff = off - off % kAioAlignment;
  const int64_t alen = ((off + len - aoff) + kAioAlignment - 1) / kAioAlignment * kAioAlignment;
  uint8_t* bounce = (uint8_t*)aligned_alloc_io((size_t)alen);
  aio_->read(fd, aoff, alen, bounce, [this, bounce, off, aoff, len, ack, done, path](int64_t r) mutable {
    release_fd(path);
    if (r < off - aoff + len) {
      aligned_free_io(bounce);
      ack.status = -6;
      ack.error = "short read";
      return done(ack, Bytes{});
    }
    bytes_ += len;
    Bytes b;
    b.ptr = bounce + (off - aoff);
    b.release = [bounce] { aligned_free_io(bounce); };
    done(ack, std::move(b));
  });
}

}  // namespace uda
