// uda_mof_supplier: a node's MOFSupplier as a process of its own (the NodeManager aux service /
// TaskTracker side, src/MOFServer/MOFSupplierMain.cc:87-143). Four roles:
//
//   uda_mof_supplier --daemon-fd N
//       the node daemon a provider front end starts (csrc/service/node_daemon.h): the node's HBM store
//       of MOF files and its merge service, driven over the control socket N
//   uda_mof_supplier mode=frontend mof_dir=D [port=P] [-Dkey=value]...
//       a NodeManager stand-in: the provider front end (uda_start as MOFSupplier through the C ABI) whose
//       getPathUda resolves map outputs in Hadoop's layout, D/<map attempt>/file.out + file.out.index (the
//       IndexCache + LocalDirAllocator lookup of the real plugin); the configuration is the -D keys and
//       nothing else, so with none it runs the library's defaults (TCP, node daemon on a GPU node). This
//       process never touches a GPU
//   uda_mof_supplier mode=mapgen mof_dir=D maps=.. reducers=.. records_per_map=.. [workload=..]
//       a map phase: generates TeraGen-shaped map outputs on the GPU, writes them in Hadoop's layout under
//       D, prints the reduce tasks' commands and expected record counts, exits
//   uda_mof_supplier key=value...   (device, maps, reducers, records_per_map, round_bytes, workload,
//                                    skew, codec, port, bind, workers, seed, service)
//       a synthetic job's map outputs held in this process's HBM and served over TCP (descriptor fetches
//       answer with hipIpc handles); service=<socket path>: also the node's merge service in process
//
// After setup the serving modes print one JSON line (the port, ...; the bench mode also every reduce
// task's expected record count and commands), then serve until stdin says "exit" (or closes); "stats"
// prints the provider's stats as one JSON line.
#include <dirent.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "uda/log.h"
#include "api_bench.h"
#include "service/merge_service.h"
#include "service/node_daemon.h"
#include "uda/cmd.h"
#include "uda/ifile.h"
#include "uda/uda_bridge.h"
#include "uda/fd_table.h"

namespace {
std::string js(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += (unsigned char)c < 0x20 ? ' ' : c;
  }
  return o + "\"";
}

// ---------------------------------------------------------------------------- front end (NodeManager)
struct FrontEnd {
  std::string mof_dir;
  std::map<std::string, std::string> conf;  // the NodeManager's configuration: -D keys only
  std::mutex mu;
  std::map<std::string, std::vector<int64_t>> index_cache;  // map attempt -> its index (IndexCache)
};

int fe_conf(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
  auto* f = static_cast<FrontEnd*>(ctx);
  std::string v = dflt ? dflt : "";
  auto it = f->conf.find(key ? key : "");
  if (it != f->conf.end()) v = it->second;
  const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)std::max(0, outlen - 1));
  std::memcpy(out, v.data(), (size_t)n);
  out[n] = 0;
  return n;
}

int fe_path(void* ctx, const char*, const char* map_id, int32_t reduce_id, uda_index_record* out) {
  auto* f = static_cast<FrontEnd*>(ctx);
  const std::string dir = f->mof_dir + "/" + map_id;
  std::vector<int64_t> idx;
  {
    std::lock_guard<std::mutex> g(f->mu);
    auto it = f->index_cache.find(map_id);
    if (it != f->index_cache.end()) idx = it->second;
  }
  if (idx.empty()) {
    std::string why;
    if (!uda::read_spill_index(dir + "/file.out.index", &idx, &why)) {
      std::fprintf(stderr, "[frontend] getPathUda %s: %s\n", map_id, why.c_str());
      return -1;
    }
    std::lock_guard<std::mutex> g(f->mu);
    f->index_cache[map_id] = idx;
  }
  if (reduce_id < 0 || (size_t)(3 * reduce_id + 2) >= idx.size()) return -1;
  out->start_offset = idx[(size_t)3 * reduce_id];
  out->raw_length = idx[(size_t)3 * reduce_id + 1];
  out->part_length = idx[(size_t)3 * reduce_id + 2];
  std::snprintf(out->path, sizeof(out->path), "%s/file.out", dir.c_str());
  return 0;
}

void fe_log(void*, const char* msg, int32_t sev) {
  if (sev <= 3) std::fprintf(stderr, "[frontend] %s\n", msg);
}

int run_frontend(const std::string& mof_dir, int port, const std::map<std::string, std::string>& conf) {
  FrontEnd f;
  f.mof_dir = mof_dir;
  f.conf = conf;
  uda_callbacks cb{};
  cb.ctx = &f;
  cb.get_conf = fe_conf;
  cb.get_path = fe_path;
  cb.log = fe_log;
  const std::vector<std::string> args = {"-w", "256", "-r", std::to_string(port), "-m", "1", "-g", "/tmp", "-s", "1024"};
  std::vector<const char*> av;
  for (auto& a : args) av.push_back(a.c_str());
  uda_handle* h = uda_start(0, (int)av.size(), av.data(), 3, 0, &cb);
  if (!h) {
    std::printf("{\"error\":\"uda_start (provider) failed\"}\n");
    return 1;
  }
  std::printf("{\"port\":%d,\"provider\":%s}\n", port, uda_stats_string(h).c_str());
  std::fflush(stdout);
  for (std::string line; std::getline(std::cin, line);) {
    if (line == "exit") break;
    if (line == "stats") {
      std::printf("%s\n", uda_stats_string(h).c_str());
      std::fflush(stdout);
    } else if (line.rfind("jobover ", 0) == 0) {
      (void)uda_do_command(h, uda::form_cmd(uda::kJobOverMsg, {line.substr(8)}).c_str());
    }
  }
  (void)uda_do_command(h, uda::form_cmd(uda::kExitMsg, {}).c_str());
  uda_destroy(h);
  return 0;
}

std::string task_json(const uda::gpu::ApiTeraSortBench& b, int reducers) {
  std::string out = "\"expected\":[";
  const auto e = b.expected_records();
  for (size_t i = 0; i < e.size(); ++i) out += (i ? "," : "") + std::to_string(e[i]);
  out += "],\"commands\":[";
  for (int r = 0; r < reducers; ++r) {
    out += r ? ",[" : "[";
    const auto cmds = b.task_commands(r);
    for (size_t i = 0; i < cmds.size(); ++i) out += (i ? "," : "") + js(cmds[i]);
    out += "]";
  }
  return out + "]";
}
}  // namespace

// The node daemon inherits every descriptor its front end's process did not mark close-on-exec (a
// NodeManager JVM's listening sockets, its log files): closed before anything else runs, so the daemon
// never holds the NodeManager's ports or files open past the NodeManager.
static void close_inherited(int keep) {
  std::vector<int> fds;
  if (DIR* d = ::opendir("/proc/self/fd")) {
    while (const dirent* e = ::readdir(d)) {
      const int fd = std::atoi(e->d_name);
      if (e->d_name[0] != '.' && fd > 2 && fd != keep) fds.push_back(fd);
    }
    ::closedir(d);  // its own descriptor is in the list: closing it again below is a harmless EBADF
  }
  for (int fd : fds) ::close(fd);
}

// The daemon's first wave starts a dozen threads per hosted task; each new thread's stack is an mmap (and
// its exit an madvise) on the address-space lock, where the wave's late tasks queued for up to 90 ms
// (profiles/r6/r7_first_wave_stall.md). `n` threads started together and joined at once leave their
// stacks in glibc's stack cache (sized by the daemon's glibc.pthread.stack_cache_size tunable), from
// which the first wave's threads then take theirs without an mmap.
static void prewarm_thread_stacks(int n) {
  std::mutex mu;
  std::condition_variable cv;
  int started = 0;
  bool go = false;
  std::vector<std::thread> ts;
  for (int i = 0; i < n; ++i)
    ts.emplace_back([&] {
      std::unique_lock<std::mutex> lk(mu);
      ++started;
      cv.notify_all();
      cv.wait(lk, [&] { return go; });
    });
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return started == n; });  // all alive at once: n distinct stacks
    go = true;
    cv.notify_all();
  }
  for (auto& t : ts) t.join();
}

int main(int argc, char** argv) {
  // the node daemon a provider front end starts (node_daemon.h): its control socket is descriptor N
  if (argc == 3 && std::string(argv[1]) == "--daemon-fd") {
    const int ctl = std::atoi(argv[2]);
    close_inherited(ctl);
    uda::pregrow_fd_table();
    if (const char* e = std::getenv("UDA_DAEMON_STACKS"); !e || std::atoi(e) > 0)
      prewarm_thread_stacks(e ? std::atoi(e) : 96);
    uda::install_crash_reporter("uda node daemon");
    return uda::run_node_daemon(ctl);
  }
  uda::pregrow_fd_table();  // the front end: a socket per fetch connection, routed client connections
  uda::install_crash_reporter("uda_mof_supplier");
  uda::gpu::ApiBenchConfig c;
  c.transport = "tcp";
  c.bind_addr = "127.0.0.1";
  c.fetch = "device";
  std::string service, mode;
  std::map<std::string, std::string> dconf;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a.rfind("-D", 0) == 0) {  // -Dkey=value or -D key=value (front end configuration)
      const std::string kv = a.size() > 2 ? a.substr(2) : (i + 1 < argc ? argv[++i] : "");
      const size_t eq = kv.find('=');
      if (eq != std::string::npos) dconf[kv.substr(0, eq)] = kv.substr(eq + 1);
      continue;
    }
    const size_t eq = a.find('=');
    if (eq == std::string::npos) {
      std::fprintf(stderr, "usage: %s key=value...\n", argv[0]);
      return 2;
    }
    const std::string k = a.substr(0, eq), v = a.substr(eq + 1);
    if (k == "device") c.device = std::atoi(v.c_str());
    else if (k == "maps") c.maps = std::atoi(v.c_str());
    else if (k == "reducers") c.reducers = std::atoi(v.c_str());
    else if (k == "records_per_map") c.records_per_map = std::atoll(v.c_str());
    else if (k == "round_bytes") c.round_bytes = std::atoll(v.c_str());
    else if (k == "workload") c.workload = v;
    else if (k == "skew") c.skew = std::atof(v.c_str());
    else if (k == "codec") c.codec = v;
    else if (k == "port") c.port = std::atoi(v.c_str());
    else if (k == "bind") c.bind_addr = v;
    else if (k == "workers") c.provider_workers = std::atoi(v.c_str());
    else if (k == "seed") c.seed = std::strtoull(v.c_str(), nullptr, 0);
    else if (k == "service") service = v;
    else if (k == "mode") mode = v;
    else if (k == "mof_dir") c.mof_dir = v;
    else {
      std::fprintf(stderr, "uda_mof_supplier: unknown key %s\n", k.c_str());
      return 2;
    }
  }
  if (mode == "frontend") {
    if (c.mof_dir.empty()) {
      std::fprintf(stderr, "uda_mof_supplier mode=frontend needs mof_dir=\n");
      return 2;
    }
    return run_frontend(c.mof_dir, c.port > 0 ? c.port : 9011, dconf);
  }
  try {
    if (mode == "mapgen") {
      if (c.mof_dir.empty()) throw std::runtime_error("mode=mapgen needs mof_dir=");
      if (c.workload != "terasort" || !c.codec.empty())
        throw std::runtime_error("mode=mapgen writes uncompressed TeraSort map outputs only");
      c.start_provider = false;
      c.keep_mof_files = true;
      uda::gpu::ApiTeraSortBench b(c);
      b.setup();
      std::printf("{\"mof_dir\":%s,\"store_bytes\":%lld,%s}\n", js(c.mof_dir).c_str(), (long long)b.store_bytes(),
                  task_json(b, c.reducers).c_str());
      std::fflush(stdout);
      return 0;
    }
    std::unique_ptr<uda::MergeService> svc;  // first: the pinned rings allocated after it are shareable
    if (!service.empty()) svc = std::make_unique<uda::MergeService>(service);
    uda::gpu::ApiTeraSortBench b(c);
    b.setup();
    std::printf("{\"port\":%d,\"store_bytes\":%lld,%s}\n", b.provider_port(), (long long)b.store_bytes(),
                task_json(b, c.reducers).c_str());
    std::fflush(stdout);
    for (std::string line; std::getline(std::cin, line);) {
      if (line == "exit") break;
      if (line == "stats") {
        std::string st = b.provider_stats();
        if (svc && !st.empty() && st.back() == '}')
          st = st.substr(0, st.size() - 1) + ",\"merge_service\":" + svc->stats_json() + "}";
        std::printf("%s\n", st.c_str());
        std::fflush(stdout);
      }
    }
  } catch (const std::exception& ex) {
    std::printf("{\"error\":%s}\n", js(ex.what()).c_str());
    return 1;
  }
  return 0;
}
