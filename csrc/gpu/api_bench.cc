// TeraSort through the C ABI with HBM-resident MOFs. See api_bench.h.
#include "api_bench.h"
#include "hbm_ledger.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <atomic>
#include <thread>

#include "device_engine.h"
#include "j2c_sink.h"
#include "secgen.h"
#include "uda/codec.h"
#include "uda/cmd.h"
#include "uda/ifile.h"
#include "uda/uda_bridge.h"

namespace uda {
namespace gpu {

namespace {
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// get_conf of both roles: a fixed table (the JobConf of this benchmark job).
struct ConfTable {
  std::map<std::string, std::string> kv;
};
int conf_cb(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
  auto* t = static_cast<ConfTable*>(ctx);
  std::string v = dflt ? dflt : "";
  auto it = t->kv.find(key);
  if (it != t->kv.end()) v = it->second;
  const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)outlen - 1);
  std::memcpy(out, v.data(), (size_t)n);
  out[n] = 0;
  return n;
}

// One reduce task's host side (the ReduceTask JVM): its dataFromUda feeds the J2C consumer.
struct TaskHost {
  ConfTable* conf = nullptr;
  J2CSink* sink = nullptr;
  int reducer = 0;
  std::mutex* mu = nullptr;
  std::condition_variable* cv = nullptr;
  int* done = nullptr;
  std::string failure;
  bool finished = false;
};
// dataFromUda: the KVBuf copy; the task's walker thread walks it and reports EOF (set_on_eof)
int data_cb(void* ctx, const void* buf, int32_t len) {
  auto* t = static_cast<TaskHost*>(ctx);
  return t->sink->consume(t->reducer, static_cast<const uint8_t*>(buf), len);
}
void failure_cb(void* ctx, const char* reason) {
  auto* t = static_cast<TaskHost*>(ctx);
  std::lock_guard<std::mutex> g(*t->mu);
  t->failure = reason ? reason : "failure";
  if (!t->finished) {
    t->finished = true;
    ++*t->done;
  }
  t->cv->notify_all();
}
int task_conf_cb(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
  return conf_cb(static_cast<TaskHost*>(ctx)->conf, key, dflt, out, outlen);
}
void log_cb(void*, const char* msg, int32_t sev) {
  if (sev <= 2) std::fprintf(stderr, "[uda api] %s\n", msg);
}

struct ProviderCtx {
  ConfTable* conf;
  const ApiTeraSortBench* bench;
};
int provider_conf_cb(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
  return conf_cb(static_cast<ProviderCtx*>(ctx)->conf, key, dflt, out, outlen);
}
int provider_path_cb(void* ctx, const char*, const char* map_id, int32_t reduce_id, uda_index_record* out) {
  int64_t rec[3];
  std::string path;
  if (!static_cast<ProviderCtx*>(ctx)->bench->resolve(map_id, reduce_id, rec, &path)) return -1;
  out->start_offset = rec[0];
  out->raw_length = rec[1];
  out->part_length = rec[2];
  std::snprintf(out->path, sizeof(out->path), "%s", path.c_str());
  return 0;
}

ConfTable& bench_conf(const ApiBenchConfig& c) {
  static ConfTable t;
  t.kv = {{"mapred.uda.transport", c.transport},
          {"mapred.uda.loopback.host", "*"},
          {"mapred.uda.merge.backend", "gpu"},
          {"mapred.uda.gpu.fetch", c.fetch},
          {"mapred.uda.gpu.device", std::to_string(c.device)},
          {"mapred.uda.kv.buf.size", std::to_string(c.kv_buf_bytes)},
          {"mapred.uda.gpu.round.bytes", std::to_string(c.round_bytes)},
          {"mapred.uda.provider.bind.address", c.bind_addr},
          // this benchmark measures the in-process shapes (bench.py --api --node runs the node daemon)
          {"mapred.uda.daemon", "0"},
          {"mapred.uda.gpu.merge.service", "off"}};
  if (c.provider_workers > 0) t.kv["mapred.uda.provider.workers"] = std::to_string(c.provider_workers);
  if (c.max_concurrent_merges >= 0) t.kv["mapred.uda.gpu.max.concurrent.merges"] = std::to_string(c.max_concurrent_merges);
  if (c.provider_hbm_bytes > 0) {
    t.kv["mapred.uda.provider.hbm.bytes"] = std::to_string(c.provider_hbm_bytes);
    t.kv["mapred.uda.provider.hbm.devices"] = std::to_string(c.device);
  }
  // A/B runs: UDA_API_CONF="key=value,key=value" adds or overrides job configuration keys
  if (const char* extra = std::getenv("UDA_API_CONF")) {
    std::string all(extra);
    size_t b = 0;
    while (b < all.size()) {
      size_t e = all.find(',', b);
      if (e == std::string::npos) e = all.size();
      const std::string kv = all.substr(b, e - b);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos && eq > 0) t.kv[kv.substr(0, eq)] = kv.substr(eq + 1);
      b = e + 1;
    }
  }
  return t;
}

std::vector<const char*> cargs(const std::vector<std::string>& v) {
  std::vector<const char*> out;
  for (auto& s : v) out.push_back(s.c_str());
  return out;
}
}  // namespace

ApiTeraSortBench::ApiTeraSortBench(const ApiBenchConfig& cfg) : cfg_(cfg) {}

ApiTeraSortBench::~ApiTeraSortBench() {
  if (provider_) {
    uda_handle* h = static_cast<uda_handle*>(provider_);
    (void)uda_do_command(h, form_cmd(kExitMsg, {}).c_str());
    uda_destroy(h);
  }
  delete static_cast<ProviderCtx*>(provider_ctx_);
  if (!cfg_.keep_mof_files)
    for (auto& kv : file_path_) {
      ::unlink(kv.second.c_str());
      ::unlink((kv.second + ".index").c_str());
      const size_t slash = kv.second.rfind('/');
      if (slash != std::string::npos) ::rmdir(kv.second.substr(0, slash).c_str());
    }
}

bool ApiTeraSortBench::resolve(const std::string& map, int reduce, int64_t rec[3], std::string* path) const {
  auto it = file_index_.find(map);
  if (it == file_index_.end() || reduce < 0 || (size_t)(3 * reduce + 2) >= it->second.size()) return false;
  for (int k = 0; k < 3; ++k) rec[k] = it->second[(size_t)(3 * reduce + k)];
  *path = file_path_.at(map);
  return true;
}

std::string ApiTeraSortBench::provider_stats() const {
  if (!provider_) return "{}";
  return uda_stats_string(static_cast<uda_handle*>(provider_));
}

int64_t ApiTeraSortBench::store_bytes() const {
  if (sec_store_) return sec_store_bytes_;
  return gen_ ? gen_->store_bytes() : 0;
}

std::vector<int64_t> ApiTeraSortBench::local_partition_records() const {
  if (cfg_.workload == "secondary") return sec_part_records_;
  return gen_ ? gen_->local_dest_records() : std::vector<int64_t>();
}

std::string ApiTeraSortBench::map_id(int global_map) const {
  char id[96];
  std::snprintf(id, sizeof(id), "attempt_%s_m_%06d_0", cfg_.job.c_str() + 4, global_map);
  return id;
}

void ApiTeraSortBench::setup() {
  if (cfg_.world < 1 || cfg_.rank < 0 || cfg_.rank >= cfg_.world) throw std::runtime_error("api bench: bad rank/world");
  if (cfg_.world > 1 && cfg_.transport != "tcp") throw std::runtime_error("api bench: world > 1 needs the tcp transport");
  // map phase stand-in: `maps` MOFs x (world * reducers) total-order partitions in this rank's HBM
  const int P = cfg_.world * cfg_.reducers;
  if (cfg_.workload == "secondary") {
    setup_secondary();
    return;
  }
  if (cfg_.workload != "terasort") throw std::runtime_error("api bench: unknown workload " + cfg_.workload);
  ShuffleConfig sc;
  sc.device = cfg_.device;
  sc.world = P;              // partitions per MOF (no exchange is ever run on this job)
  sc.rank = cfg_.rank;       // seeds the rank's maps
  sc.maps_per_rank = cfg_.maps;
  sc.records_per_map = cfg_.records_per_map;
  sc.seed = cfg_.seed;
  sc.deliver_host = false;
  gen_.reset(new ShuffleJob(sc));
  gen_->generate();
  if (cfg_.world == 1) expected_ = gen_->local_dest_records();
  // MOFSupplier handle (TaskTracker / NodeManager side)
  uda_handle* h = nullptr;
  if (cfg_.start_provider) {
    ConfTable& conf = bench_conf(cfg_);
    auto* pctx = new ProviderCtx{&conf, this};
    provider_ctx_ = pctx;
    uda_callbacks cb{};
    cb.ctx = pctx;
    cb.get_conf = provider_conf_cb;
    cb.get_path = provider_path_cb;
    cb.log = log_cb;
    const std::vector<std::string> args = {"-w", "256", "-r", std::to_string(cfg_.port > 0 ? cfg_.port : 9011),
                                           "-m", "1", "-g", "/tmp", "-s", "1024"};
    auto av = cargs(args);
    h = uda_start(0, (int)av.size(), av.data(), 2, 0, &cb);
    if (!h) throw std::runtime_error("api bench: uda_start (provider) failed");
    provider_ = h;
  } else if (cfg_.mof_dir.empty() || !cfg_.codec.empty()) {
    throw std::runtime_error("api bench: a map phase without a provider writes uncompressed MOF files (mof_dir)");
  }
  map_ids_.clear();
  for (int m = 0; m < cfg_.maps; ++m) {
    const std::string id = map_id(cfg_.rank * cfg_.maps + m);
    map_ids_.push_back(id);
    std::vector<int64_t> index;
    for (int r = 0; r < P; ++r) {
      const auto ir = gen_->index_record(m, r);
      index.insert(index.end(), ir.begin(), ir.end());
    }
    if (!cfg_.mof_dir.empty()) {
      // the map task's output in Hadoop's layout, <dir>/<attempt>/file.out + file.out.index (the provider
      // finds it through getPathUda: IndexCache + LocalDirAllocator in Hadoop)
      const std::string dir = cfg_.mof_dir + "/" + id;
      if (::mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST)
        throw std::runtime_error("api bench: cannot create " + dir + ": " + strerror(errno));
      const std::string path = dir + "/file.out";
      write_spill_index(path + ".index", index);
      const int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_CLOEXEC, 0644);
      if (fd < 0) throw std::runtime_error("api bench: cannot create " + path + ": " + strerror(errno));
      const int64_t len = gen_->mof_bytes(m);
      std::vector<uint8_t> buf((size_t)std::min<int64_t>(len, 256ll << 20));
      for (int64_t off = 0; off < len;) {
        const int64_t n = std::min<int64_t>((int64_t)buf.size(), len - off);
        HIP_CHECK(hipMemcpy(buf.data(), gen_->mof_device_ptr(m) + off, (size_t)n, hipMemcpyDeviceToHost));
        for (int64_t w = 0; w < n;) {
          const ssize_t r = ::pwrite(fd, buf.data() + w, (size_t)(n - w), off + w);
          if (r <= 0) {
            ::close(fd);
            throw std::runtime_error("api bench: write to " + path + " failed");
          }
          w += r;
        }
        off += n;
      }
      (void)::fdatasync(fd);
      ::close(fd);
      file_index_[id] = index;
      file_path_[id] = path;
      continue;
    }
    if (cfg_.host_mofs) {  // a map output in host memory (page cache / local disk stand-in)
      host_mofs_.emplace_back((size_t)gen_->mof_bytes(m));
      HIP_CHECK(hipMemcpy(host_mofs_.back().data(), gen_->mof_device_ptr(m), (size_t)gen_->mof_bytes(m),
                          hipMemcpyDeviceToHost));
      if (uda_provider_register_mof(h, cfg_.job.c_str(), id.c_str(), host_mofs_.back().data(), gen_->mof_bytes(m),
                                    index.data(), P) != 0)
        throw std::runtime_error(std::string("api bench: register_mof failed: ") + uda_last_error(h));
      continue;
    }
    if (!cfg_.codec.empty()) continue;  // registered compressed below
    if (uda_provider_register_mof_device(h, cfg_.job.c_str(), id.c_str(), gen_->mof_device_ptr(m), gen_->mof_bytes(m),
                                         index.data(), P, cfg_.device) != 0)
      throw std::runtime_error(std::string("api bench: register_mof_device failed: ") + uda_last_error(h));
  }
  if (!cfg_.codec.empty()) compress_store();
  // the generated store served only as the map side's output: the compressed copy (codec) or the
  // MOF files (mof_dir) are what the provider serves, so its HBM goes back to the reduce tasks
  if (!cfg_.codec.empty() || !cfg_.mof_dir.empty() || cfg_.host_mofs) gen_->release_store();
}

// Compressed map outputs (what a job with mapred.compress.map.output writes): each partition of each
// MOF is block-compressed on the host and the compressed MOFs are packed into one HBM store,
// registered as device MOFs with index {offset, raw length, compressed length}. Sized for the
// flagship scale (130 GB per GPU): the raw MOFs go to host memory once and leave HBM, each MOF is
// compressed partition by partition into its own host region (compressed data never outgrows the
// raw bytes it replaces; checked), and only then is the compressed store allocated -- raw and
// compressed copies never share HBM, and the host holds one copy plus a partition per thread.
void ApiTeraSortBench::compress_store() {
  const Codec c = cfg_.codec == "snappy" ? Codec::kSnappy : cfg_.codec == "lzo" ? Codec::kLzo : Codec::kNone;
  if (c == Codec::kNone) throw std::runtime_error("api bench: unknown codec " + cfg_.codec);
  const int P = cfg_.world * cfg_.reducers, M = cfg_.maps;
  std::vector<int64_t> raw_off((size_t)M + 1, 0);
  for (int m = 0; m < M; ++m) raw_off[(size_t)m + 1] = raw_off[(size_t)m] + gen_->mof_bytes(m);
  std::unique_ptr<uint8_t[]> host_mem(new uint8_t[(size_t)std::max<int64_t>(raw_off[(size_t)M], 1)]);  // no zero fill
  uint8_t* host = host_mem.get();
  for (int m = 0; m < M; ++m)
    HIP_CHECK(hipMemcpy(host + raw_off[(size_t)m], gen_->mof_device_ptr(m), (size_t)gen_->mof_bytes(m),
                        hipMemcpyDeviceToHost));
  gen_->release_store();
  std::vector<int64_t> comp_len((size_t)M, 0);
  std::vector<std::vector<int64_t>> idx((size_t)M);
  std::vector<std::thread> ts;
  std::mutex emu;
  std::string err;
  const int nt = std::max(1, std::min<int>({M, 16, (int)std::thread::hardware_concurrency()}));
  for (int t = 0; t < nt; ++t)
    ts.emplace_back([&, t] {
      try {
        for (int m = t; m < M; m += nt) {
          uint8_t* mof = host + raw_off[(size_t)m];
          int64_t at = 0;  // compressed bytes written back into the MOF's own region
          for (int r = 0; r < P; ++r) {
            const auto ir = gen_->index_record(m, r);  // {offset, raw, part}
            const std::vector<uint8_t> b = block_compress(c, mof + ir[0], (size_t)ir[2], 256 << 10);
            if (at + (int64_t)b.size() > ir[0] + ir[2])
              throw std::runtime_error("compressed partition outgrew its raw bytes (incompressible input)");
            std::memmove(mof + at, b.data(), b.size());
            idx[(size_t)m].insert(idx[(size_t)m].end(), {at, ir[2], (int64_t)b.size()});
            at += (int64_t)b.size();
          }
          comp_len[(size_t)m] = at;
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(emu);
        err = e.what();
      }
    });
  for (auto& t : ts) t.join();
  if (!err.empty()) throw std::runtime_error("api bench: compressing the MOFs: " + err);
  std::vector<int64_t> off((size_t)M + 1, 0);
  for (int m = 0; m < M; ++m) off[(size_t)m + 1] = off[(size_t)m] + (comp_len[(size_t)m] + 255) / 256 * 256;
  comp_store_.reset(new DeviceBuffer((size_t)std::max<int64_t>(off[(size_t)M], 16), /*resident=*/true));
  uda_handle* h = static_cast<uda_handle*>(provider_);
  for (int m = 0; m < M; ++m) {
    uint8_t* dst = comp_store_->as<uint8_t>() + off[(size_t)m];
    HIP_CHECK(hipMemcpy(dst, host + raw_off[(size_t)m], (size_t)comp_len[(size_t)m], hipMemcpyHostToDevice));
    const std::string id = map_id(cfg_.rank * M + m);
    if (uda_provider_register_mof_device(h, cfg_.job.c_str(), id.c_str(), dst, comp_len[(size_t)m],
                                         idx[(size_t)m].data(), P, cfg_.device) != 0)
      throw std::runtime_error(std::string("api bench: register_mof_device failed: ") + uda_last_error(h));
    comp_bytes_ += comp_len[(size_t)m];
  }
}

// Secondary-sort map outputs (secgen.h) generated straight into one HBM store and registered as
// device MOFs: the reduce tasks take the generic-key device merge (key-range rounds).
void ApiTeraSortBench::setup_secondary() {
  HIP_CHECK(hipSetDevice(cfg_.device));
  // partitions of every rank's maps: world x reducers; reduce task 0 of every rank is the hot one
  const int P = cfg_.world * cfg_.reducers;
  const SecGenPlan plan = secgen_plan(cfg_.maps, P, cfg_.records_per_map, cfg_.skew,
                                      cfg_.seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)cfg_.rank), cfg_.reducers);
  sec_store_bytes_ = plan.store_bytes();
  sec_store_.reset(new DeviceBuffer((size_t)sec_store_bytes_, /*resident=*/true));
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  secgen_write(plan, sec_store_->as<uint8_t>(), s);
  HIP_CHECK(hipStreamDestroy(s));
  sec_part_records_.assign((size_t)P, 0);
  for (int m = 0; m < cfg_.maps; ++m)
    for (int q = 0; q < P; ++q) sec_part_records_[(size_t)q] += plan.nrec[(size_t)m * P + q];
  if (cfg_.world == 1) expected_ = sec_part_records_;
  ConfTable& conf = bench_conf(cfg_);
  auto* pctx = new ProviderCtx{&conf, this};
  provider_ctx_ = pctx;
  uda_callbacks cb{};
  cb.ctx = pctx;
  cb.get_conf = provider_conf_cb;
  cb.get_path = provider_path_cb;
  cb.log = log_cb;
  const std::vector<std::string> args = {"-w", "256", "-r", std::to_string(cfg_.port > 0 ? cfg_.port : 9011),
                                         "-m", "1", "-g", "/tmp", "-s", "1024"};
  auto av = cargs(args);
  uda_handle* h = uda_start(0, (int)av.size(), av.data(), 2, 0, &cb);
  if (!h) throw std::runtime_error("api bench: uda_start (provider) failed");
  provider_ = h;
  map_ids_.clear();
  for (int m = 0; m < cfg_.maps; ++m) {
    const std::string id = map_id(cfg_.rank * cfg_.maps + m);
    map_ids_.push_back(id);
    std::vector<int64_t> index;
    int64_t off = 0;
    for (int q = 0; q < P; ++q) {
      const int64_t b = plan.part_bytes[(size_t)m * P + q];
      index.insert(index.end(), {off, b, b});
      off += b;
    }
    const uint8_t* base = sec_store_->as<uint8_t>() + plan.mof_off[(size_t)m];
    const int64_t len = plan.mof_off[(size_t)m + 1] - plan.mof_off[(size_t)m];
    if (uda_provider_register_mof_device(h, cfg_.job.c_str(), id.c_str(), base, len, index.data(), P, cfg_.device) != 0)
      throw std::runtime_error(std::string("api bench: register_mof_device failed: ") + uda_last_error(h));
  }
}

std::vector<std::string> ApiTeraSortBench::task_commands(int r) const {
  const int R = cfg_.reducers, W = cfg_.world;
  const int g = cfg_.rank * R + r;  // the job's reduce task index
  char rt[96];
  std::snprintf(rt, sizeof(rt), "attempt_%s_r_%06d_0", cfg_.job.c_str() + 4, g);
  const std::string codec_cls = cfg_.codec == "snappy" ? "org.apache.hadoop.io.compress.SnappyCodec"
                                : cfg_.codec == "lzo"  ? "com.hadoop.compression.lzo.LzoCodec"
                                                       : "null";
  std::vector<std::string> out;
  const std::vector<std::string> init = {std::to_string(W * cfg_.maps), cfg_.job, rt, "0", std::to_string(1 << 20),
                                         std::to_string(16 << 10), "org.apache.hadoop.io.Text", codec_cls,
                                         std::to_string(256 << 10), "0", "0"};
  out.push_back(form_cmd(kInitMsg, init));
  // rotating rank order: the tasks of rank d start with rank d + 1's maps, spreading the load
  for (int k = 0; k < W; ++k) {
    const int p = (cfg_.rank + 1 + k) % W;
    const std::string host = W == 1 ? (cfg_.transport == "tcp" ? "127.0.0.1" : "localhost") : peers_[(size_t)p];
    for (int m = 0; m < cfg_.maps; ++m) {
      const std::vector<std::string> f = {host, cfg_.job, map_id(p * cfg_.maps + m), std::to_string(g)};
      out.push_back(form_cmd(kFetchMsg, f));
    }
  }
  return out;
}

int ApiTeraSortBench::provider_port() const {
  if (!provider_) return -1;
  const std::string st = uda_stats_string(static_cast<uda_handle*>(provider_));
  const char* js = st.c_str();
  const char* q = std::strstr(js, "\"port\":");
  return q ? std::atoi(q + 7) : -1;
}

std::map<std::string, double> ApiTeraSortBench::step(bool validate, std::string* info) {
  const int R = cfg_.reducers;
  const int W = cfg_.world;
  if ((int)expected_.size() != R) throw std::runtime_error("api bench: expected record counts not set");
  if (W > 1 && (int)peers_.size() != W) throw std::runtime_error("api bench: provider addresses not set");
  std::mutex mu;
  std::condition_variable cv;
  int done = 0;
  std::vector<TaskHost> hosts(R);  // before the sink: its reduce-task threads report EOF into them
  J2CSink sink(R, cfg_.kv_buf_bytes, J2CSink::plugin_threaded());
  sink.set_on_eof([&hosts](int r) {  // the reduce task's thread walked its EOF marker
    TaskHost& t = hosts[(size_t)r];
    std::lock_guard<std::mutex> g(*t.mu);
    if (!t.finished) {
      t.finished = true;
      ++*t.done;
    }
    t.cv->notify_all();
  });
  sink.set_check_order(validate);
  sink.set_key_kind(1);  // Text: content order (TeraSort's fixed keys order the same either way)
  // device-wide HBM in use, sampled through the step (the peak includes the map-output store)
  HbmLedger::get().reset_peak(cfg_.device);  // the ledger's peak of this step alone
  std::atomic<bool> sampling{true};
  std::atomic<int64_t> peak_used{0};
  std::thread sampler([&] {
    (void)hipSetDevice(cfg_.device);
    while (sampling.load()) {
      size_t free_b = 0, total_b = 0;
      if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
        peak_used.store(std::max<int64_t>(peak_used.load(), (int64_t)(total_b - free_b)));
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  });
  struct SamplerGuard {
    std::atomic<bool>& on;
    std::thread& t;
    ~SamplerGuard() {
      on = false;
      if (t.joinable()) t.join();
    }
  } sampler_guard{sampling, sampler};
  ConfTable& conf = bench_conf(cfg_);
  std::vector<uda_handle*> handles(R, nullptr);
  std::vector<std::string> errors(R);
  const double t0 = now_ms();
  // every reduce task is its own "JVM" thread driving its handle: start, INIT, FETCH per map
  std::vector<std::thread> ts;
  for (int r = 0; r < R; ++r) {
    ts.emplace_back([&, r] {
      TaskHost& th = hosts[r];
      th.conf = &conf;
      th.sink = &sink;
      th.reducer = r;
      th.mu = &mu;
      th.cv = &cv;
      th.done = &done;
      uda_callbacks cb{};
      cb.ctx = &th;
      cb.data_from_uda = data_cb;
      cb.get_conf = task_conf_cb;
      cb.failure = failure_cb;
      cb.log = log_cb;
      const std::vector<std::string> args = {"-w", "256", "-r", std::to_string(cfg_.port > 0 ? cfg_.port : 9011),
                                             "-a", "1", "-m", "1", "-g", "/tmp", "-s", "1024"};
      auto av = cargs(args);
      uda_handle* h = uda_start(1, (int)av.size(), av.data(), 2, 0, &cb);
      handles[r] = h;
      auto fail = [&](const std::string& why) {
        std::lock_guard<std::mutex> g(mu);
        errors[r] = why;
        if (!th.finished) {
          th.finished = true;
          ++done;
        }
        cv.notify_all();
      };
      if (!h) return fail("uda_start failed");
      for (const std::string& c : task_commands(r))
        if (uda_do_command(h, c.c_str()) != 0) return fail(uda_last_error(h));
    });
  }
  for (auto& t : ts) t.join();
  {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(900), [&] { return done == R; }))
      throw std::runtime_error("api bench: reduce tasks did not finish within 900 s");
  }
  const double t1 = now_ms();
  std::string paths;
  double max_ws = 0, max_rounds = 0, hbm_wait_sum = 0, hbm_wait_max = 0, task_total_max = 0;
  for (int r = 0; r < R; ++r) {
    if (!handles[r]) continue;
    (void)uda_reduce_exit(handles[r]);  // joins the merge thread: its stats are final after this
    const std::string st = uda_stats_string(handles[r]);
    const char* js = st.c_str();
    if (st.size() > 2) {
      if (r == 0) paths = st;
      auto num = [&](const char* key) {
        const char* q = std::strstr(js, key);
        return q ? std::atof(q + std::strlen(key)) : 0.0;
      };
      max_ws = std::max(max_ws, num("\"gpu_ws_bytes\":"));
      max_rounds = std::max(max_rounds, num("\"rpq_rounds\":"));
      const double wait = num("\"hbm_wait_ms\":"), total = num("\"total_ms\":");
      hbm_wait_sum += wait;
      hbm_wait_max = std::max(hbm_wait_max, wait);
      task_total_max = std::max(task_total_max, total);
    }
    uda_destroy(handles[r]);
  }
  sink.flush();  // every delivered KVBuf walked
  sampling = false;
  if (sampler.joinable()) sampler.join();
  const double t2 = now_ms();
  for (int r = 0; r < R; ++r) {
    if (!errors[r].empty()) throw std::runtime_error("reduce task " + std::to_string(r) + ": " + errors[r]);
    if (!hosts[r].failure.empty()) throw std::runtime_error("reduce task " + std::to_string(r) + " failed: " + hosts[r].failure);
    if (sink.error(r) != 0) throw std::runtime_error("reduce task " + std::to_string(r) + ": consumer framing error");
    if (sink.records(r) != expected_[r])
      throw std::runtime_error("reduce task " + std::to_string(r) + ": consumer parsed " + std::to_string(sink.records(r)) +
                               " records, expected " + std::to_string(expected_[r]));
  }
  std::map<std::string, double> out;
  double bytes = 0, recs = 0, bufs = 0, oerr = 0;
  for (int r = 0; r < R; ++r) {
    bytes += (double)sink.bytes(r);
    recs += (double)sink.records(r);
    bufs += (double)sink.buffers(r);
    oerr += (double)sink.order_errors(r);
  }
  out["wall_ms"] = t1 - t0;
  out["close_ms"] = t2 - t1;
  out["bytes"] = bytes;
  out["records"] = recs;
  out["buffers"] = bufs;
  out["order_errors"] = validate ? oerr : -1;
  out["peak_hbm_bytes"] = (double)peak_used.load();
  {
    const HbmLedger::Stats ls = HbmLedger::get().stats(cfg_.device);
    out["hbm_budget_bytes"] = (double)ls.budget;
    out["hbm_ledger_peak_bytes"] = (double)ls.peak;
    out["hbm_budget_waits"] = (double)ls.waits;
    out["hbm_over_budget_bytes"] = (double)ls.over;  // allocations outside a reservation past the budget
  }
  out["max_task_ws_bytes"] = max_ws;
  out["max_task_rounds"] = max_rounds;
  out["hbm_wait_ms_sum"] = hbm_wait_sum;  // the tasks' budget waits this step
  out["hbm_wait_ms_max"] = hbm_wait_max;
  out["task_total_ms_max"] = task_total_max;
  if (info) *info = paths;
  return out;
}

}  // namespace gpu
}  // namespace uda
