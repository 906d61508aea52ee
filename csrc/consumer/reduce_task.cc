#include "reduce_task.h"
#include "uda/fault.h"

#include <fcntl.h>
#include <climits>
#include <cstdlib>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <iomanip>
#include <random>
#include <sstream>

#include "../gpu/hbm_ledger.h"
#include "uda/log.h"
#include "uda/node_registry.h"
#include "uda/queues.h"
#include "uda/safe_file.h"
#include "uda/trace.h"
#include "uda/thread_name.h"

namespace uda {

namespace {
constexpr int kProgressReportLimit = 20;  // PROGRESS_REPORT_LIMIT (MergeManager.cc:44)
constexpr int kExtraBuffers = 10;         // EXTRA_RDMA_BUFFERS (reducer.cc:50)
constexpr int kMinParallelLpqs = 3;       // MIN_PARALLEL_LPQS (MergeManager.h:125)

// free text in the stats (error reasons): escaped and capped, so the object stays one short JSON line
std::string json_escape(const std::string& in, size_t cap = 512) {
  std::string o;
  for (char c : in.size() > cap ? in.substr(0, cap) : in) {
    if (c == '"' || c == '\\') o += '\\';
    o += (unsigned char)c < 0x20 ? ' ' : c;
  }
  return o;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Merged-records spill file reader for the RPQ (SuperSegment, StreamRW.cc:813-861).
struct FileSource {
  int fd = -1;
  int64_t off = 0;
  int64_t read(uint8_t* dst, int64_t cap) {
    for (;;) {
      ssize_t r = ::pread(fd, dst, (size_t)cap, off);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) throw UdaError(std::string("spill read failed: ") + strerror(errno));
      off += r;
      return r;
    }
  }
};
}  // namespace

// --------------------------------------------------------------------------------- MofFetcher
MofFetcher::MofFetcher(ReduceTask* task, FetchParams p, int64_t buf_size, Codec codec)
    : task_(task), p_(std::move(p)), buf_size_(buf_size), codec_(codec) {
  bufs_[0].resize((size_t)buf_size_);
  bufs_[1].resize((size_t)buf_size_);
  proto_.job_id = p_.job_id;
  proto_.map_id = p_.map_id;
  proto_.reduce_id = p_.reduce_id;
  if (codec_ != Codec::kNone) dec_ = std::make_unique<BlockDecoder>(codec_);
}

void MofFetcher::start() {
  std::function<void()> call;
  {
    std::lock_guard<std::mutex> g(mu_);
    call = prepare(0);
  }
  call();
}

std::function<void()> MofFetcher::prepare(int b) {
  FetchRequest req = proto_;
  req.fetched = requested_;
  req.buf_len = buf_size_;
  requested_ += buf_size_;
  inflight_[b] = true;
  ready_[b] = false;
  auto self = shared_from_this();
  uint8_t* dst = bufs_[b].data();
  return [self, b, req, dst] {
    ReduceTask* t = self->task_;
    t->fetch_begin();  // the task outlives every completion: exit() waits for fetch_end
    t->transport()->fetch(self->p_.host, req, dst, [self, b, t](const FetchAck& a) {
      self->on_done(b, a);
      t->fetch_end();
    });
  };
}

void MofFetcher::on_done(int b, const FetchAck& a) {
  bool first = false;
  {
    std::unique_lock<std::mutex> lk(mu_, std::defer_lock);
    lk.lock();
    inflight_[b] = false;
    if (a.status != 0) {
      error_ = a.error.empty() ? "fetch failed" : a.error;
    } else {
      len_[b] = a.sent;
      ready_[b] = true;
      part_len_ = a.part_len;
      proto_.mof_offset = a.mof_offset;
      proto_.raw_len = a.raw_len;
      proto_.part_len = a.part_len;
      proto_.path = a.path;
    }
    if (!first_done_) {
      first_done_ = true;
      first = true;
    }
    cv_.notify_all();  // under the lock: a woken consumer may drop the last reference
  }
  if (first) {
    {
      std::lock_guard<std::mutex> g(task_->mu_);
      task_->fetched_.push_back(shared_from_this());
    }
    task_->cv_.notify_all();
  }
}

int64_t MofFetcher::pull_raw(uint8_t* dst, int64_t cap) {
  std::unique_lock<std::mutex> lk(mu_);
  if (part_len_ >= 0 && consumed_ >= part_len_) {
    lk.unlock();
    release_pair();
    return 0;
  }
  const int b = cur_;
  auto t0 = std::chrono::steady_clock::now();
  cv_.wait(lk, [&] { return ready_[b] || !error_.empty(); });
  wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  if (!error_.empty()) throw UdaError("fetch of " + p_.map_id + " failed: " + error_);
  const int64_t n = std::min(len_[b], cap);
  std::memcpy(dst, bufs_[b].data(), (size_t)n);
  consumed_ += n;
  ready_[b] = false;
  cur_ ^= 1;
  // keep one request ahead: the buffer just drained and the other one (if idle) get the next
  // chunks in offset order
  const int nb = cur_;  // next chunk expected here
  std::vector<std::function<void()>> calls;
  if (!inflight_[nb] && !ready_[nb] && requested_ < part_len_) calls.push_back(prepare(nb));
  if (!inflight_[b] && !ready_[b] && requested_ < part_len_) calls.push_back(prepare(b));
  const bool ended = consumed_ >= part_len_;
  lk.unlock();
  for (auto& c : calls) c();
  {
    std::lock_guard<std::mutex> g(task_->st_mu_);
    task_->st_.bytes_fetched += n;
  }
  if (ended) release_pair();
  return n;
}

int64_t MofFetcher::take_first(uint8_t* dst, int64_t cap) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return ready_[0] || !error_.empty(); });
  if (!error_.empty()) throw UdaError("fetch of " + p_.map_id + " failed: " + error_);
  const int64_t n = std::min(len_[0], cap);
  std::memcpy(dst, bufs_[0].data(), (size_t)n);
  consumed_ = n;
  ready_[0] = false;
  lk.unlock();
  {
    std::lock_guard<std::mutex> g(task_->st_mu_);
    task_->st_.bytes_fetched += n;
  }
  release_pair();
  return n;
}

int64_t ReduceTask::fetch_direct(const FetchParams& f, uint8_t* dst, int64_t off, int64_t end, int depth,
                                 const std::function<void(int64_t, int64_t)>& on_prefix, int64_t prefix_step) {
  std::mutex m;
  std::condition_variable c;
  int inflight = 0;
  std::string err;
  int64_t next = off;
  // landed-prefix tracking (requests complete out of order): [off, prefix) has landed, `done` holds
  // the later completed requests, [reported, prefix) has not been handed to on_prefix yet
  std::map<int64_t, int64_t> done;
  int64_t prefix = off, reported = off;
  auto landed = [&](int64_t at, int64_t len) {  // m held
    if (!on_prefix) return;
    done[at] = len;
    for (auto it = done.begin(); it != done.end() && it->first == prefix; it = done.erase(it)) prefix += it->second;
    if (prefix - reported >= std::max<int64_t>(prefix_step, 1) || prefix == end) {
      on_prefix(reported, prefix);
      reported = prefix;
    }
  };
  auto issue = [&](int64_t at) {
    FetchRequest req;
    req.job_id = f.job_id;
    req.map_id = f.map_id;
    req.reduce_id = f.reduce_id;
    req.fetched = at;
    req.buf_len = std::min(direct_chunk_, end - at);
    const int64_t want = req.buf_len;
    fetch_begin();
    const int64_t ti = trace::host_enabled() ? trace::now_ns() : 0;
    transport_->fetch(f.host, req, dst + at, [&, want, at, ti](const FetchAck& a) {
      if (ti) trace::host_event("fetch_req", want, (int64_t)(uintptr_t)(dst + at), ti, trace::now_ns());
      std::lock_guard<std::mutex> g(m);
      if (a.status != 0 && err.empty()) err = a.error.empty() ? "fetch failed" : a.error;
      if (a.status == 0 && a.sent != want && err.empty()) err = "short fetch";
      if (err.empty()) landed(at, want);
      --inflight;
      c.notify_all();
      fetch_end();
    });
  };
  std::unique_lock<std::mutex> lk(m);
  for (;;) {
    while (next < end && inflight < depth && err.empty() && !stop_) {
      const int64_t at = next;
      next += std::min(direct_chunk_, end - at);
      ++inflight;
      lk.unlock();
      issue(at);  // a transport may complete inline
      lk.lock();
    }
    const bool can_issue = next < end && err.empty() && !stop_;
    if (!can_issue && inflight == 0) break;
    c.wait(lk, [&] { return inflight == 0 || (can_issue && inflight < depth); });
  }
  if (!err.empty()) throw UdaError("fetch of " + f.map_id + " failed: " + err);
  if (next < end) throw UdaError("reduce task stopped during fetch");
  lk.unlock();
  std::lock_guard<std::mutex> g(st_mu_);
  st_.bytes_fetched += end - off;
  return end;
}

void MofFetcher::release_pair() {
  if (released_.exchange(true)) return;  // buffers go back to the pool once
  {
    std::lock_guard<std::mutex> g(task_->mu_);
    task_->free_pairs_++;
  }
  task_->cv_.notify_all();
}

int64_t MofFetcher::pull(uint8_t* dst, int64_t cap) {
  if (!dec_) return pull_raw(dst, cap);
  std::vector<uint8_t> tmp;
  for (;;) {
    size_t r = dec_->read(dst, (size_t)cap);
    if (r > 0) return (int64_t)r;
    if (tmp.empty()) tmp.resize((size_t)buf_size_);
    int64_t n = pull_raw(tmp.data(), (int64_t)tmp.size());
    if (n == 0) {
      if (!dec_->idle()) throw UdaError("compressed MOF ended inside a block");
      return 0;
    }
    dec_->feed(tmp.data(), (size_t)n);
  }
}

// --------------------------------------------------------------------------------- ReduceTask
ReduceTask::ReduceTask(const NetlevOptions& net, Host* host) : net_(net), host_(host) {}

ReduceTask::~ReduceTask() { exit(); }

void ReduceTask::handle(const HadoopCmd& cmd) {
  std::string err;
  switch (cmd.header) {
    case kInitMsg: {
      InitParams p;
      if (!parse_init_params(cmd, &p, &err)) throw ProtocolError(err);
      on_init(p);
      break;
    }
    case kFetchMsg: {
      FetchParams f;
      if (!parse_fetch_params(cmd, &f, &err)) throw ProtocolError(err);
      {
        std::lock_guard<std::mutex> g(mu_);
        ++fetch_cmds_;
      }
      if (!restored_tasks_.empty()) {
        // restored LPQs are matched by map *task*: a re-executed map (new attempt id) must not be
        // merged next to the LPQ that already holds its old attempt's records
        auto it = restored_tasks_.find(map_task_of(f.map_id));
        if (it != restored_tasks_.end()) {
          if (it->second == f.map_id) {  // already merged into a checkpointed LPQ
            UDA_LOG(kDebug, "fetch of %s skipped: restored from the LPQ checkpoint", f.map_id.c_str());
            break;
          }
          const std::string had = it->second;
          discard_checkpoint();
          throw UdaError("map task re-executed since the LPQ checkpoint (" + had + " -> " + f.map_id +
                         "): checkpoint discarded, the next attempt starts clean");
        }
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        fetch_list_.push_back(f);
      }
      cv_.notify_all();
      break;
    }
    case kFinalMsg: {
      std::lock_guard<std::mutex> g(mu_);
      final_ = true;
      cv_.notify_all();
      break;
    }
    case kExitMsg:
      exit();
      break;
    default:
      UDA_LOG(kDebug, "ignoring command %d", (int)cmd.header);
      break;
  }
}

std::string sandbox_check_dir(const std::vector<std::string>& roots, const std::string& p) {
  char buf[PATH_MAX];
  if (!::realpath(p.c_str(), buf)) return p + ": " + strerror(errno);
  const std::string c(buf);
  for (const auto& r : roots) {
    if (r.empty()) continue;
    if (c == r || (c.size() > r.size() && c.compare(0, r.size(), r) == 0 && (r.back() == '/' || c[r.size()] == '/')))
      return "";
  }
  return p + " is outside the node's local directories";
}

bool sandbox_trusted_file(const std::vector<std::string>& dirs, const std::string& path) {
  if (!owned_regular_file(path)) return false;
  if (dirs.empty()) return true;
  const size_t slash = path.rfind('/');
  if (slash == std::string::npos) return false;
  return sandbox_check_dir(dirs, path.substr(0, slash == 0 ? 1 : slash)).empty();
}

void ReduceTask::on_init(const InitParams& p_in) {
  if (inited_) throw ProtocolError("INIT received twice");
  InitParams p = p_in;
  if (sandbox_.enabled) {
    // a task run for another local user: its id names files, and its local dirs are where this
    // process's user creates, reads back and unlinks them
    if (p.reduce_task_id.empty() || p.reduce_task_id.find("..") != std::string::npos ||
        p.reduce_task_id.find_first_not_of("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789_.-") !=
            std::string::npos)
      throw ProtocolError("reduce task id '" + p.reduce_task_id + "' is not allowed for a confined task");
    std::vector<std::string> canon;
    for (const auto& d : p.local_dirs) {
      const std::string why = sandbox_check_dir(sandbox_.roots, d);
      if (!why.empty()) throw ProtocolError("confined task: local dir " + why);
      char buf[PATH_MAX];
      canon.push_back(::realpath(d.c_str(), buf) ? std::string(buf) : d);
    }
    p.local_dirs = canon;
  }
  init_ = p;
  kind_ = key_kind_from_class(p.key_class.c_str());
  if (kind_ == KeyKind::kUnsupported)
    throw ProtocolError("using compare function for unsupported type: " + p.key_class);
  bool unsup = false;
  codec_ = codec_from_class(p.codec, &unsup);
  if (unsup) throw ProtocolError("unsupported compression codec: " + p.codec);
  const int maps = p.num_maps;
  // LPQ geometry (reduce_task::init, reducer.cc:260-285)
  if (p.lpq_size > 0) {
    num_lpqs_ = maps / p.lpq_size;
    if (maps % p.lpq_size > 1) num_lpqs_++;
  } else {
    num_lpqs_ = (int)std::sqrt((double)maps);
  }
  num_parallel_lpqs_ = std::max<int>(kMinParallelLpqs, (int)host_->conf_i64("mapred.rdma.num.parallel.lpqs", 0));
  const bool hybrid = net_.online == 2 && num_lpqs_ > 1 && maps >= num_lpqs_;
  const int max_mofs_in_lpq = num_lpqs_ > 0 ? maps / num_lpqs_ + 1 : maps;
  num_kv_bufs_ = hybrid ? max_mofs_in_lpq * num_parallel_lpqs_ : std::max(1, maps);
  // buffer sizing (handle_init_msg, reducer.cc:102-120)
  int64_t max_buf = std::min<int64_t>(p.max_buf_bytes, net_.buf_size > 0 ? net_.buf_size : p.max_buf_bytes);
  if (max_buf <= 0) max_buf = 1 << 20;
  if (p.shuffle_mem_bytes > 0 && p.shuffle_mem_bytes < (int64_t)num_kv_bufs_ * max_buf * 2) {
    max_buf = p.shuffle_mem_bytes / ((int64_t)num_kv_bufs_ * 2);
    if (max_buf < p.min_buf_bytes) throw UdaError("Not enough memory for rdma buffers");
    UDA_LOG(kWarn, "using calculated buffer size %ld instead of %ld", (long)max_buf, (long)p.max_buf_bytes);
  }
  const int64_t page = sysconf(_SC_PAGESIZE);
  buffer_size_ = max_buf - max_buf % page;
  if (buffer_size_ <= 0 || buffer_size_ < p.min_buf_bytes) throw UdaError("RDMA Buffer is too small");
  free_pairs_ = num_kv_bufs_ + kExtraBuffers;
  fetch_buf_ = buffer_size_;
  int64_t uncomp_buf = buffer_size_;
  if (codec_ != Codec::kNone) {
    // compressed: the pair's 2*buffer_size is split between the fetch side and the decoded side
    // (reducer.cc:463-491): the decoded side gets at least one codec block plus a minimal fetch
    // buffer, then `mapred.rdma.compression.buffer.ratio` of what is left, plus anything the fetch
    // side would get above mapred.rdma.buf.size.
    if (codec_ == Codec::kLzo) {
      const std::string v = host_->get_conf("io.compression.codec.lzo.decompressor", "LZO1X");
      if (v != "LZO1X" && v != "LZO1X_SAFE" && v != "LZO1X_ASM" && v != "LZO1X_ASM_SAFE" &&
          v != "LZO1X_ASM_FAST" && v != "LZO1X_ASM_FAST_SAFE")
        throw UdaError("unsupported io.compression.codec.lzo.decompressor " + v +
                       " (the in-tree and device decoders read the LZO1X stream format)");
    }
    const double ratio = std::atof(host_->get_conf("mapred.rdma.compression.buffer.ratio", "0.20").c_str());
    const int64_t max_fetch = host_->conf_i64("mapred.rdma.buf.size", 1024) * 1024;
    const int64_t min_fetch = p.min_buf_bytes;
    const int64_t hard_min = p.comp_block_size + min_fetch;
    const int64_t pair = buffer_size_ * 2;
    if (pair < hard_min + min_fetch) {
      // the reference gives up here ("not enough memory to allocate buffers"); our decoders keep
      // their own block-sized output, so a small pair still works with the whole pair fetching
      UDA_LOG(kWarn, "buffer pair %ld < codec block %ld + 2 x min buffer %ld: no split, fetch chunk %ld",
              (long)pair, (long)p.comp_block_size, (long)min_fetch, (long)buffer_size_);
    } else {
    const int64_t delta = pair - (hard_min + min_fetch);
    uncomp_buf = hard_min + (int64_t)((double)delta * std::min(1.0, std::max(0.0, ratio)));
    fetch_buf_ = pair - uncomp_buf;
    const int64_t spare = std::max<int64_t>(fetch_buf_ - max_fetch, 0);
    fetch_buf_ -= spare;
    uncomp_buf += spare;
    }
  }
  if (fault_hit("HOST_ALLOC")) throw UdaError("injected allocation failure for the fetch buffer pool");
  kv_buf_size_ = host_->conf_i64("mapred.uda.kv.buf.size", 1 << 20);
  fault_spec_ = host_->get_conf("mapred.uda.fault.inject", "");
  // fetches straight into a partition-sized destination (the GPU staged path) are not bound to the
  // double-buffer size: larger requests mean fewer answers to frame and dispatch per byte
  direct_chunk_ = std::max<int64_t>(buffer_size_, host_->conf_i64("mapred.uda.fetch.request.bytes", 4 << 20));
  // "auto" (default): the GPU merge when this process sees a HIP device, else the CPU (reference) merge
  backend_ = host_->get_conf("mapred.uda.merge.backend", "auto");
  if (backend_ == "auto") {
    backend_ = gpu::visible_device_keys().empty() ? "cpu" : "gpu";
    UDA_LOG(kInfo, "mapred.uda.merge.backend=auto: %s merge", backend_.c_str());
  }
  if (backend_ != "cpu" && backend_ != "gpu") throw ProtocolError("unknown mapred.uda.merge.backend " + backend_);
  // the reference's consumer always fetches over the network from the providers (RdmaClient,
  // src/Merger/reducer.cc:412-437); loopback only reaches a provider in this very process
  const std::string tr = host_->get_conf("mapred.uda.transport", "tcp");
  transport_ = (tr == "loopback") ? make_loopback_client()
                                  : make_tcp_client(net_.data_port, net_.wqes_per_conn,
                                                    (int)host_->conf_i64("mapred.uda.tcp.connections", 4));
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.backend = backend_;
    st_.fetch_buf_bytes = fetch_buf_;
    st_.uncomp_buf_bytes = uncomp_buf;
  }
  inited_ = true;
  UDA_LOG(kInfo, "reduce task %s: maps=%d approach=%d lpqs=%d kv_bufs=%d buffer=%ld codec=%s key=%s backend=%s",
          p.reduce_task_id.c_str(), maps, net_.online, num_lpqs_, num_kv_bufs_, (long)buffer_size_,
          codec_name(codec_), key_kind_name(kind_), backend_.c_str());
  // CPU: the hybrid (approach 2) LPQ files; GPU: the disk-tier LPQ spills of the GPU hybrid merge
  checkpoint_ = host_->conf_i64("mapred.uda.lpq.checkpoint", 0) != 0 && (backend_ == "gpu" || net_.online == 2);
  if (checkpoint_ && sandbox_.enabled && init_.local_dirs.empty()) checkpoint_ = false;  // no /tmp manifests
  if (checkpoint_) load_checkpoint();
  if (backend_ == "gpu") {
    device_conf_ = host_->get_conf("mapred.uda.gpu.device", "auto");
    hbm_budget_conf_ = std::atof(host_->get_conf("mapred.uda.gpu.hbm.budget", "0").c_str());
  }
  if (backend_ == "gpu" && host_->conf_i64("mapred.uda.gpu.prewarm", 1) != 0) {
    PrewarmConf pc;
    pc.early_h2d = host_->conf_i64("mapred.uda.gpu.early.h2d", 1) != 0;
    // pinned fetch-arena blocks, not for tasks that only fetch device descriptors
    if (host_->get_conf("mapred.uda.gpu.fetch", "auto") != "device")
      pc.pinned_bytes = host_->conf_i64("mapred.uda.gpu.prewarm.pinned.mb", 1024) << 20;
    pc.round_bytes = host_->conf_i64("mapred.uda.gpu.round.bytes", 2ll << 30);
    pc.maps = p.num_maps;
    prewarm_thr_ = std::thread([this, pc] { name_thread("uda-task-warm"); prewarm_gpu(pc); });
  }
  merge_thr_ = std::thread([this] { name_thread("uda-task-merge"); merge_main(); });
}

void ReduceTask::place_on_gpu() {
  const std::string conf = forced_device_ >= 0 ? std::to_string(forced_device_) : device_conf_;
  const std::vector<std::string> keys = gpu::visible_device_keys();
  if (keys.empty()) {
    device_ = 0;  // merge_gpu reports "no HIP device" when the task gets there
    return;
  }
  NodeRegistry* reg = NodeRegistry::instance();
  if (conf != "auto" && !conf.empty()) {
    device_ = std::atoi(conf.c_str());
    if (device_ < 0 || device_ >= (int)keys.size())
      throw UdaError("mapred.uda.gpu.device=" + conf + " but " + std::to_string(keys.size()) + " GPU(s) are visible");
    if (reg) registry_slot_ = reg->add_task(keys[(size_t)device_], init_.reduce_task_id);
  } else if (reg) {
    const NodeRegistry::Placement pl = reg->place_task(keys, init_.reduce_task_id);
    device_ = pl.index;
    registry_slot_ = pl.slot;
  } else {
    device_ = 0;
  }
  // per-device HBM budget: bytes, or a fraction of the device's HBM (default 0.92)
  gpu::HbmLedger::get().configure(device_, hbm_budget_conf_);
  std::lock_guard<std::mutex> g(st_mu_);
  st_.gpu_device = device_;
}

// attempt_<jt>_<job>_m_<task>_<n> -> attempt_<jt>_<job>_m_<task> (the map task, any attempt)
std::string map_task_of(const std::string& attempt) {
  const size_t u = attempt.rfind('_');
  if (u != std::string::npos && u + 1 < attempt.size() &&
      attempt.find_first_not_of("0123456789", u + 1) == std::string::npos)
    return attempt.substr(0, u);
  return attempt;
}

// The manifest and every LPQ file it lists are removed; nothing of the failed attempt is reused. The
// in-memory lists stay as they are: this runs on the host's command thread while the merge thread may
// be reading them, and the task is failing anyway (the next attempt starts from the missing manifest).
void ReduceTask::discard_checkpoint() {
  for (const auto& f : restored_files_) {
    ::unlink(f.c_str());
    ::unlink((f + ".idx").c_str());
  }
  ::unlink(checkpoint_path().c_str());
}

std::string ReduceTask::checkpoint_path() const {
  // keyed by job + partition, not by attempt: attempt_<job>_r_<part>_<n> -> drop "_<n>"
  std::string key = init_.reduce_task_id;
  const size_t u = key.rfind('_');
  if (u != std::string::npos && u + 1 < key.size() &&
      key.find_first_not_of("0123456789", u + 1) == std::string::npos)
    key.resize(u);
  const std::string dir = init_.local_dirs.empty() ? std::string("/tmp") : init_.local_dirs[0];
  return dir + "/uda." + key + ".lpq.manifest";
}

// Manifest lines: "lpq <index> <bytes> <path> <map_id,map_id,...>". An entry is taken only if it
// continues the LPQ sequence, its file exists with that size and it holds the MOF count the LPQ
// geometry gives that index (same num_maps / lpq_size as the failed attempt).
void ReduceTask::load_checkpoint() {
  // only a manifest this process's user wrote, listing files it wrote (in a confined task: inside its
  // local dirs); anything else is not ours to read back or unlink
  const std::vector<std::string> trust_dirs = sandbox_.enabled ? init_.local_dirs : std::vector<std::string>();
  if (!sandbox_trusted_file(trust_dirs, checkpoint_path())) return;
  std::ifstream in(checkpoint_path());
  if (!in) return;
  const int maps = init_.num_maps;
  if (backend_ == "gpu") {  // "glpq <index> <bytes> <path> <ids>": groups are budget-sized, no geometry
    std::string line;
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::string tag, path, ids;
      int idx = -1;
      long long bytes = -1;
      if (!(ls >> tag >> idx >> bytes >> path >> ids) || tag != "glpq") break;
      struct stat sb, si;
      if (idx != (int)restored_files_.size() || ::stat(path.c_str(), &sb) != 0 || (long long)sb.st_size != bytes ||
          ::stat((path + ".idx").c_str(), &si) != 0 || !sandbox_trusted_file(trust_dirs, path) ||
          !sandbox_trusted_file(trust_dirs, path + ".idx"))
        break;
      std::set<std::string> v;
      for (size_t b = 0;;) {
        const size_t e = ids.find(',', b);
        v.insert(ids.substr(b, e == std::string::npos ? std::string::npos : e - b));
        if (e == std::string::npos) break;
        b = e + 1;
      }
      restored_files_.push_back(path);
      restored_maps_.insert(v.begin(), v.end());
    }
    if ((int)restored_maps_.size() > maps) {  // not this job's shape: start over
      restored_files_.clear();
      restored_maps_.clear();
    }
    for (const auto& m : restored_maps_) restored_tasks_[map_task_of(m)] = m;
    if (!restored_files_.empty())
      UDA_LOG(kInfo, "GPU LPQ checkpoint: resuming with %zu LPQs (%zu MOFs)", restored_files_.size(),
              restored_maps_.size());
    return;
  }
  if (num_lpqs_ <= 1 || maps < num_lpqs_) return;
  const int per = maps / num_lpqs_;
  const int regular = num_lpqs_ - maps % num_lpqs_;
  std::string line;
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    std::string tag, path, ids;
    int idx = -1;
    long long bytes = -1;
    if (!(ls >> tag >> idx >> bytes >> path >> ids) || tag != "lpq") break;
    const int want = (idx < regular) ? per : per + 1;
    struct stat sb;
    if (idx != (int)restored_files_.size() || ::stat(path.c_str(), &sb) != 0 || (long long)sb.st_size != bytes ||
        !sandbox_trusted_file(trust_dirs, path))
      break;
    std::vector<std::string> v;
    for (size_t b = 0; b <= ids.size();) {
      const size_t e = ids.find(',', b);
      v.push_back(ids.substr(b, e == std::string::npos ? std::string::npos : e - b));
      if (e == std::string::npos) break;
      b = e + 1;
    }
    if ((int)v.size() != want) break;
    restored_files_.push_back(path);
    restored_maps_.insert(v.begin(), v.end());
  }
  for (const auto& m : restored_maps_) restored_tasks_[map_task_of(m)] = m;
  if (!restored_files_.empty())
    UDA_LOG(kInfo, "LPQ checkpoint: resuming with %zu LPQs (%zu MOFs) from %s", restored_files_.size(),
            restored_maps_.size(), checkpoint_path().c_str());
}

void ReduceTask::exit() {
  exiting_ = true;
  stop_ = true;
  cv_.notify_all();
  if (merge_thr_.joinable()) merge_thr_.join();
  if (prewarm_thr_.joinable()) prewarm_thr_.join();
  if (transport_) transport_->close();
  // completions of requests still in flight (a provider worker may be serving one) touch this task
  std::unique_lock<std::mutex> lk(inflight_mu_);
  if (!inflight_cv_.wait_for(lk, std::chrono::seconds(120), [&] { return inflight_ == 0; }))
    UDA_LOG(kError, "reduce task exit: %ld fetch completions still outstanding", (long)inflight_);
  lk.unlock();
  if (registry_slot_ >= 0) {
    if (NodeRegistry* reg = NodeRegistry::instance()) reg->release(registry_slot_);
    registry_slot_ = -1;
  }
}

void ReduceTask::fetch_begin() {
  std::lock_guard<std::mutex> g(inflight_mu_);
  ++inflight_;
}

void ReduceTask::fetch_end() {
  // notify under the lock: once exit() sees zero it may destroy the task (and this cv)
  std::lock_guard<std::mutex> g(inflight_mu_);
  --inflight_;
  inflight_cv_.notify_all();
}

void ReduceTask::merge_main() {
  auto t0 = std::chrono::steady_clock::now();
  FaultScope faults(fault_spec_);  // this task's own injected faults (mapred.uda.fault.inject)
  try {
    const std::string gfetch = host_->get_conf("mapred.uda.gpu.fetch", "auto");  // auto | device | host
    // a resumed attempt (LPQ checkpoint of an earlier staged attempt) merges its restored runs on the
    // staged path: the device path has no notion of restored maps (their FETCHes are dropped)
    // compressed map outputs decode on the device straight from the descriptors (F6); hybrid-mode
    // tasks need no LPQ spills when the partitions stay in the provider's HBM (the merge runs in
    // key-range rounds that bound its working set), so both take the device path when the first
    // answers are device descriptors
    const bool dev_codec = codec_ == Codec::kNone || host_->conf_i64("mapred.uda.gpu.decompress", 1) != 0;
    if (backend_ == "gpu" && dev_codec && gfetch != "host" && restored_files_.empty() &&
        merge_gpu_device(gfetch == "auto")) {
      // done: partitions merged where the provider holds them
    } else if (backend_ == "gpu") {
      merge_gpu();
    }
    else if (net_.online == 2)
      merge_hybrid();
    else
      merge_online();
  } catch (const std::exception& e) {
    // stop_ alone also means "an internal failure stopped the fetchers": only a host-requested
    // exit() silences the report
    if (!exiting_) host_->fail(e.what());
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.total_ms = ms_since(t0);
  }
  finished_ = true;
}

std::unique_ptr<Segment> ReduceTask::segment_for(std::shared_ptr<MofFetcher> f, int index) {
  auto seg = std::make_unique<StreamSegment>(
      [f](uint8_t* dst, int64_t cap) { return f->pull(dst, cap); }, buffer_size_);
  seg->index = index;
  return seg;
}

void ReduceTask::fetch_phase(MergeQueue* q, int n, std::vector<std::string>* map_ids) {
  std::mt19937_64 rng((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count());
  int sent = 0, inserted = 0;
  std::vector<FetchParams> pending;
  while (inserted < n) {
    std::vector<std::shared_ptr<MofFetcher>> to_start, arrived;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] {
        return stop_ || !fetched_.empty() ||
               ((!fetch_list_.empty() || !pending.empty()) && free_pairs_ > 0 && sent < n);
      });
      if (stop_) throw UdaError("reduce task stopped during fetch");
      // random fetch order spreads load over providers (list_shuffle_in_vector, UdaUtil.h:56-101)
      while (!fetch_list_.empty()) {
        pending.push_back(fetch_list_.front());
        fetch_list_.pop_front();
      }
      std::shuffle(pending.begin(), pending.end(), rng);
      while (!pending.empty() && free_pairs_ > 0 && sent < n) {
        to_start.push_back(std::make_shared<MofFetcher>(this, pending.back(), fetch_buf_, codec_));
        pending.pop_back();
        free_pairs_--;
        sent++;
      }
      while (!fetched_.empty()) {
        arrived.push_back(fetched_.front());
        fetched_.pop_front();
      }
    }
    for (auto& f : to_start) f->start();
    for (auto& f : arrived) {
      if (map_ids) map_ids->push_back(f->params().map_id);
      q->insert(segment_for(f, next_index_++));
      inserted++;
      total_count_++;
      progress_count_++;
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.maps_fetched++;
      }
      if (progress_count_ == kProgressReportLimit || total_count_ == init_.num_maps) {
        host_->fetch_over();
        progress_count_ = 0;
      }
    }
  }
  // requests not needed by this phase go back to the shared list (hybrid: next LPQ)
  if (!pending.empty()) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& p : pending) fetch_list_.push_front(p);
  }
}

void ReduceTask::merging_phase(MergeQueue* q) {
  std::vector<uint8_t> buf((size_t)kv_buf_size_);
  KVWriter w(q);
  bool done = false;
  while (!done) {
    if (stop_) throw UdaError("reduce task stopped during merge");
    int64_t len = 0;
    done = w.fill(buf.data(), (int64_t)buf.size(), &len);
    if (host_->data_from_uda(buf.data(), (int32_t)len) != 0) throw UdaError("dataFromUda callback failed");
    std::lock_guard<std::mutex> g(st_mu_);
    st_.buffers++;
    st_.bytes_delivered += len;
  }
  std::lock_guard<std::mutex> g(st_mu_);
  st_.records += w.records();
}

void ReduceTask::merge_online() {
  auto t0 = std::chrono::steady_clock::now();
  MergeQueue q(kind_);
  fetch_phase(&q, init_.num_maps);
  const double f = ms_since(t0);
  merging_phase(&q);
  std::lock_guard<std::mutex> g(st_mu_);
  st_.fetch_ms = f;
  st_.merge_ms = ms_since(t0) - f;
}

void ReduceTask::merge_hybrid() {
  const int maps = init_.num_maps;
  if (num_lpqs_ <= 1 || maps < num_lpqs_) return merge_online();
  const int per = maps / num_lpqs_;
  const int regular = num_lpqs_ - maps % num_lpqs_;
  std::vector<std::string> dirs = init_.local_dirs;
  if (dirs.empty()) dirs.push_back("/tmp");
  std::mt19937 rng((unsigned)std::chrono::steady_clock::now().time_since_epoch().count());
  int dir_counter = (int)(rng() % dirs.size());
  ExternalQuotaQueue<std::pair<MergeQueue*, std::string>> pending((size_t)num_parallel_lpqs_);
  std::exception_ptr fetch_err;
  auto t0 = std::chrono::steady_clock::now();
  const int first = (int)restored_files_.size();  // LPQs restored from a checkpoint
  std::mutex ids_mu;
  std::map<std::string, std::vector<std::string>> lpq_ids;  // spill path -> its MOFs
  if (first > 0) {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.restored_lpqs = first;
    st_.restored_maps = (int64_t)restored_maps_.size();
    st_.maps_fetched += (int64_t)restored_maps_.size();
  }
  total_count_ += (int)restored_maps_.size();
  if (first > 0 && total_count_ == maps) host_->fetch_over();
  // LPQ fetcher thread (fetch_lpqs, MergeManager.cc:202-232)
  std::thread fetcher([&] {
    try {
      for (int i = first; i < num_lpqs_; ++i) {
        const int n = (i < regular) ? per : per + 1;
        const std::string& dir = dirs[(size_t)(++dir_counter) % dirs.size()];
        char name[64];
        snprintf(name, sizeof(name), ".lpq-%03d", i);
        std::string path = dir + "/uda." + init_.reduce_task_id + name;
        pending.wait_and_reserve();
        auto* q = new MergeQueue(kind_);
        std::vector<std::string> ids;
        fetch_phase(q, n, checkpoint_ ? &ids : nullptr);
        {
          std::lock_guard<std::mutex> g(ids_mu);
          lpq_ids[path] = std::move(ids);
        }
        pending.push_reserved({q, path});
      }
    } catch (...) {
      fetch_err = std::current_exception();
      pending.push_reserved({nullptr, std::string()});
    }
  });
  std::vector<std::string> files = restored_files_;
  size_t checkpointed = files.size();  // files[0, checkpointed) are listed in the manifest
  const std::string manifest = checkpoint_ ? checkpoint_path() : std::string();
  if (checkpoint_ && first == 0) ::unlink(manifest.c_str());  // stale or unusable: start over
  auto discard = [&] {  // failure: keep what the manifest lists when checkpointing
    for (size_t k = checkpoint_ ? checkpointed : 0; k < files.size(); ++k) ::unlink(files[k].c_str());
  };
  std::vector<uint8_t> buf((size_t)kv_buf_size_);
  try {
    for (int i = first; i < num_lpqs_; ++i) {
      auto item = pending.wait_and_pop_without_dereserve();
      if (!item.first) break;
      std::unique_ptr<MergeQueue> q(item.first);
      // LPQ merge -> spill file (write_kv_to_file, StreamRW.cc:863-887): records + EOF marker
      int fd = create_private_file(item.second, O_WRONLY);
      if (fd < 0) throw UdaError("cannot create spill file " + item.second + ": " + strerror(errno));
      files.push_back(item.second);
      KVWriter w(q.get());
      bool done = false;
      int64_t written = 0;
      while (!done) {
        int64_t len = 0;
        done = w.fill(buf.data(), (int64_t)buf.size(), &len);
        const int64_t body = done ? len - kEofBytes : len;  // EOF once, at the very end
        if (body > 0 && ::write(fd, buf.data(), (size_t)body) != body) {
          ::close(fd);
          throw UdaError("spill write failed");
        }
        written += body;
      }
      const uint8_t eof[2] = {0xFF, 0xFF};
      if (::write(fd, eof, 2) != 2) {
        ::close(fd);
        throw UdaError("spill write failed");
      }
      if (checkpoint_) {
        // durable before it is listed: a resumed attempt trusts every manifest entry
        if (::fsync(fd) != 0) {
          ::close(fd);
          throw UdaError("spill fsync failed");
        }
        std::string ids;
        {
          std::lock_guard<std::mutex> g(ids_mu);
          for (const auto& m : lpq_ids[item.second]) ids += (ids.empty() ? "" : ",") + m;
        }
        if (!append_owned_line(manifest, "lpq " + std::to_string(i) + " " + std::to_string(written + 2) + " " +
                                              item.second + " " + ids)) {
          ::close(fd);
          throw UdaError("cannot append to LPQ manifest " + manifest);
        }
        checkpointed = files.size();
      }
      ::close(fd);
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.lpqs++;
        st_.spill_bytes += written + 2;
      }
      pending.dereserve();
      if (fault_hit("LPQ_DONE")) throw UdaError("injected failure after an LPQ spill");
    }
  } catch (...) {
    stop_ = true;
    cv_.notify_all();
    pending.dereserve();
    fetcher.join();
    discard();
    throw;
  }
  fetcher.join();
  if (fetch_err) {
    discard();
    std::rethrow_exception(fetch_err);
  }
  const double fetch_ms = ms_since(t0);
  // RPQ over the spilled LPQ outputs (SuperSegment)
  MergeQueue rpq(kind_);
  std::vector<std::shared_ptr<FileSource>> srcs;
  for (size_t i = 0; i < files.size(); ++i) {
    auto s = std::make_shared<FileSource>();
    s->fd = ::open(files[i].c_str(), O_RDONLY | O_CLOEXEC);
    if (s->fd < 0) throw UdaError("cannot reopen spill file " + files[i]);
    srcs.push_back(s);
    auto seg = std::make_unique<StreamSegment>([s](uint8_t* d, int64_t c) { return s->read(d, c); },
                                               std::max<int64_t>(buffer_size_, 1 << 20));
    seg->index = (int)i;
    rpq.insert(std::move(seg));
  }
  merging_phase(&rpq);
  for (auto& s : srcs) ::close(s->fd);
  for (auto& f : files) ::unlink(f.c_str());  // transient, like SuperSegment's dtor
  if (checkpoint_) ::unlink(manifest.c_str());
  std::lock_guard<std::mutex> g(st_mu_);
  st_.fetch_ms = fetch_ms;
  st_.merge_ms = ms_since(t0) - fetch_ms;
}

ReduceStats ReduceTask::stats() const {
  std::lock_guard<std::mutex> g(st_mu_);
  return st_;
}

std::string ReduceTask::stats_json() const {
  ReduceStats s = stats();
  std::ostringstream o;
  o << "{\"role\":\"net_merger\",\"backend\":\"" << s.backend << "\",\"maps_fetched\":" << s.maps_fetched
    << ",\"bytes_fetched\":" << s.bytes_fetched << ",\"bytes_delivered\":" << s.bytes_delivered
    << ",\"records\":" << s.records << ",\"buffers\":" << s.buffers << ",\"lpqs\":" << s.lpqs
    << ",\"spill_bytes\":" << s.spill_bytes << ",\"fetch_ms\":" << s.fetch_ms << ",\"merge_ms\":" << s.merge_ms
    << ",\"total_ms\":" << s.total_ms << ",\"device_decoded_blocks\":" << s.device_decoded_blocks
    << ",\"rpq_rounds\":" << s.rpq_rounds << ",\"hybrid_direct\":" << s.hybrid_direct << ",\"merge_budget_from_ledger\":" << s.merge_budget_from_ledger << ",\"gpu_h2d_ms\":" << s.gpu_h2d_ms
    << ",\"gpu_device_ms\":" << s.gpu_device_ms << ",\"gpu_d2h_wait_ms\":" << s.gpu_d2h_wait_ms
    << ",\"gpu_sink_ms\":" << s.gpu_sink_ms << ",\"gpu_decode_ms\":" << s.gpu_decode_ms << ",\"gpu_gate_wait_ms\":" << s.gpu_gate_wait_ms << ",\"gpu_prewarm_ms\":" << s.gpu_prewarm_ms << ",\"gpu_prewarm_wait_ms\":" << s.gpu_prewarm_wait_ms << ",\"gpu_prewarm_phases\":\"" << json_escape(s.gpu_prewarm_phases) << "\"" << ",\"fetch_buf_bytes\":" << s.fetch_buf_bytes
    << ",\"uncomp_buf_bytes\":" << s.uncomp_buf_bytes << ",\"restored_lpqs\":" << s.restored_lpqs
    << ",\"restored_maps\":" << s.restored_maps << ",\"device_descriptors\":" << s.device_descriptors << ",\"unmapped_descriptors\":" << s.unmapped_descriptors << ",\"unmapped_reason\":\"" << json_escape(s.unmapped_reason) << "\"" << ",\"descriptor_map_ms\":" << s.descriptor_map_ms << ",\"fetch_cmd_wait_ms\":" << s.fetch_cmd_wait_ms << ",\"fetch_ack_wait_ms\":" << s.fetch_ack_wait_ms << ",\"merge_start_boot_ms\":" << std::fixed << std::setprecision(1) << s.merge_start_boot_ms << ",\"fetch_sent_boot_ms\":" << s.fetch_sent_boot_ms << std::defaultfloat << std::setprecision(6) << ",\"first_data_ms\":" << s.first_data_ms << ",\"gpu_ws_bytes\":" << s.gpu_ws_bytes
    << ",\"host_fetched_bytes\":" << s.host_fetched_bytes << ",\"local_read_bytes\":" << s.local_read_bytes << ",\"hbm_wait_ms\":" << s.hbm_wait_ms
    << ",\"hbm_reserved\":" << s.hbm_reserved << ",\"round_bytes\":" << s.round_bytes << ",\"gpu_device\":" << s.gpu_device << ",\"merge_path\":\"" << s.merge_path << "\""
    << ",\"finished\":" << (finished_ ? "true" : "false") << "}";
  return o.str();
}

}  // namespace uda
