// C ABI of libuda.so (see uda/uda_bridge.h). Role dispatch mirrors Java_..._startNative
// (src/UdaBridge.cc:187-263): is_net_merger selects the NetMerger (ReduceTask) or the MOFSupplier.
#include "uda/uda_bridge.h"

#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../consumer/reduce_task.h"
#include "../gpu/hbm_ledger.h"
#include "../provider/supplier.h"
#include "../service/merge_service.h"
#include "../service/node_daemon.h"
#include "uda/cmd.h"
#include "uda/host.h"
#include "uda/log.h"
#include "uda/fd_table.h"

#define UDA_VERSION_STRING "uda_amd-0.1.0 (MI355X-native; reference API 3.4.1)"

struct uda_handle {
  bool is_merger = false;
  uda::NetlevOptions opt;
  std::unique_ptr<uda::Host> host;
  std::unique_ptr<uda::Supplier> supplier;
  std::unique_ptr<uda::ReduceTask> task;
  std::unique_ptr<uda::RemoteReduceTask> remote;  // NetMerger hosted by the node's merge service
  std::unique_ptr<uda::MergeService> service;     // provider without a node daemon: an explicit in-process service
  std::shared_ptr<uda::NodeDaemonSet> daemon;  // provider: the node daemons (HBM store + merge service), one per GPU
  std::string last_error;
  std::mutex mu;
};

namespace {
std::mutex g_log_mu;
uda_callbacks g_log_cb;  // the most recent handle's log sink (the logger is process-wide)
bool g_log_cb_set = false;

void log_trampoline(void*, const char* msg, int sev) {
  uda_callbacks cb;
  {
    std::lock_guard<std::mutex> g(g_log_mu);
    if (!g_log_cb_set) return;
    cb = g_log_cb;
  }
  if (cb.log) cb.log(cb.ctx, msg, sev);
}

int fail_call(uda_handle* h, const std::string& why) {
  h->last_error = why;
  UDA_LOG(uda::kError, "%s", why.c_str());
  return -1;
}
}  // namespace

extern "C" {

const char* uda_version(void) { return UDA_VERSION_STRING; }

void uda_set_log_level(int level) { uda::log_set_threshold(level); }

uda_handle* uda_start(int is_net_merger, int argc, const char* const* argv, int log_level, int log_to_file,
                      const uda_callbacks* cb) {
  auto h = std::make_unique<uda_handle>();
  h->is_merger = is_net_merger != 0;
  h->host = std::make_unique<uda::Host>(cb);
  uda::log_set_threshold(log_level);
  std::vector<std::string> args;
  for (int i = 0; i < argc; ++i) args.emplace_back(argv[i] ? argv[i] : "");
  std::string err;
  if (!uda::parse_options(args, &h->opt, &err)) {
    UDA_LOG(uda::kError, "bad options: %s", err.c_str());
    return nullptr;
  }
  // a JVM host: grow its descriptor table once now rather than by doublings under load, each of which
  // stalls every thread that opens a descriptor for an RCU grace period (uda/fd_table.h)
  uda::pregrow_fd_table(h->is_merger ? 1 << 14 : 1 << 17);
  if (log_to_file) {
    uda::log_open_file(h->opt.log_dir, h->is_merger ? "NetMerger" : "MOFSupplier");
  } else if (cb && cb->log) {
    std::lock_guard<std::mutex> g(g_log_mu);
    g_log_cb = *cb;
    g_log_cb_set = true;
  }
  uda::log_set_sink(log_trampoline, nullptr);  // outside g_log_mu: the logger calls us under its own lock
  // "The version is <v>" is the line the regression tools parse (tools/regression.py)
  UDA_LOG(uda::kInfo, "UDA: The version is %s role=%s", UDA_VERSION_STRING, h->is_merger ? "NetMerger" : "MOFSupplier");
  try {
    if (h->is_merger) {
      // The node merge service (in the node daemon) hosts the NetMerger where the GPU context, the pools
      // and the provider's HBM store already live (merge_service.h). Default "auto": the node's service
      // of the provider on this task's data port, if one runs; none (a node without GPUs, a provider
      // without its daemon): the task merges in this process.
      const std::string tr = h->host->get_conf("mapred.uda.transport", "tcp");
      std::string svc = h->host->get_conf("mapred.uda.gpu.merge.service", "auto");
      const bool auto_svc = svc == "auto";
      if (auto_svc) svc = tr == "tcp" ? uda::MergeService::default_path(h->opt.data_port) : std::string();
      if (svc == "off" || svc == "0" || svc == "false") svc.clear();
      if (!svc.empty()) {
        try {
          h->remote = std::make_unique<uda::RemoteReduceTask>(svc, args, h->host.get());
          UDA_LOG(uda::kInfo, "NetMerger hosted by the merge service at %s", svc.c_str());
        } catch (const std::exception& e) {
          // no service on the node is the normal case of "auto" without a GPU: not worth a warning
          const bool absent = auto_svc && std::string(e.what()).find("not reachable") != std::string::npos;
          UDA_LOG(absent ? uda::kInfo : uda::kWarn, "merge service unavailable at %s (%s): merging in this process",
                  svc.c_str(), e.what());
        }
      }
      if (!h->remote) h->task = std::make_unique<uda::ReduceTask>(h->opt, h->host.get());
    } else {
      uda::Supplier::Options so;
      so.transport = h->host->get_conf("mapred.uda.transport", "tcp");
      so.loopback_host = h->host->get_conf("mapred.uda.loopback.host", "*");
      so.bind_addr = h->host->get_conf("mapred.uda.provider.bind.address", "");
      so.io_threads = (int)h->host->conf_i64("mapred.uda.provider.blocked.threads.per.disk", 4);
      so.workers = (int)h->host->conf_i64("mapred.uda.provider.workers", 8);
      so.odirect = h->host->conf_bool("mapred.uda.provider.odirect", false);
      so.copy_serve = h->host->conf_bool("mapred.uda.provider.copy.serve", false);
      // The node daemon (node_daemon.h) holds the node's GPU state: the HBM store of MOF files and the
      // merge service. "auto": on a node with a GPU driver and the TCP transport (the loopback transport
      // only reaches reducers in this very process).
      const std::string dm = h->host->get_conf("mapred.uda.daemon", "auto");
      const bool use_daemon = so.transport == "tcp" && (dm == "1" || dm == "true" ||
                                                        (dm == "auto" && uda::NodeDaemonClient::node_has_gpu()));
      std::shared_ptr<uda::DeviceStore> local_store;
      if (!use_daemon) {
        // no daemon: the store runs in this process only when sized explicitly, the service only at an
        // explicit path (tests and benchmarks that measure the in-process shapes)
        const std::string hb = h->host->get_conf("mapred.uda.provider.hbm.bytes", "auto");
        uda::LocalStoreOptions lo;
        lo.capacity = hb == "auto" ? 0 : std::atoll(hb.c_str());
        lo.lease_s = h->host->conf_f64("mapred.uda.provider.hbm.lease.s", 600);
        lo.idle_evict_s = h->host->conf_f64("mapred.uda.provider.hbm.idle.evict.s", 30);
        lo.cached_read = h->host->conf_i64("mapred.uda.provider.hbm.cached.read", 1) != 0;
        if (lo.capacity > 0) {
          // default: stripe the store over every GPU the provider sees, so a node's reduce tasks (placed
          // over all GPUs, mapred.uda.gpu.device=auto) find their map outputs spread the same way
          std::string devs = h->host->get_conf("mapred.uda.provider.hbm.devices", "all");
          if (devs == "all") {
            devs.clear();
            const int n = (int)uda::gpu::visible_device_keys().size();
            for (int d = 0; d < n; ++d) devs += (d ? "," : "") + std::to_string(d);
            if (devs.empty()) devs = "0";
          }
          lo.devices.clear();
          for (size_t b = 0; b <= devs.size();) {
            const size_t e = devs.find(',', b);
            const std::string t = devs.substr(b, e == std::string::npos ? std::string::npos : e - b);
            if (!t.empty()) lo.devices.push_back(std::atoi(t.c_str()));
            if (e == std::string::npos) break;
            b = e + 1;
          }
          local_store = uda::make_local_device_store(lo);
          UDA_LOG(uda::kInfo, "MOFSupplier HBM store in process: %ld bytes over %zu GPU(s)", (long)lo.capacity,
                  lo.devices.size());
        }
        // before the supplier allocates its pinned rings, so they are shareable with the service's clients
        const std::string svc = h->host->get_conf("mapred.uda.gpu.merge.service", "auto");
        if (svc != "auto" && svc != "off" && svc != "0" && svc != "false" && !svc.empty())
          h->service = std::make_unique<uda::MergeService>(svc);
      }
      h->supplier = std::make_unique<uda::Supplier>(h->opt, so, h->host.get());
      if (local_store) h->supplier->set_store(local_store);
      h->supplier->start();
      if (use_daemon) {
        uda::NodeDaemonClient::Options dopt;
        dopt.exe = h->host->get_conf("mapred.uda.daemon.exe", "");
        dopt.start_args = args;
        dopt.data_port = h->supplier->port();
        dopt.start_timeout_s = h->host->conf_f64("mapred.uda.daemon.start.timeout.s", 120);
        dopt.max_restarts = (int)h->host->conf_i64("mapred.uda.daemon.restarts", 3);
        // the daemon's own stderr (HIP runtime messages, a crash's last words); its log lines go to ours
        const char* env_log = std::getenv("UDA_DAEMON_LOG");
        dopt.log_path = h->host->get_conf("mapred.uda.daemon.log",
                                          env_log ? env_log
                                                  : (h->opt.log_dir.empty() ? std::string("/tmp") : h->opt.log_dir) +
                                                        "/udaNodeDaemon.log");
        // one daemon per GPU (node_daemon.h NodeDaemonSet): a GPU's fault fails its own hosted tasks only,
        // and every GPU's tasks get their own process (HIP context, hardware queues)
        uda::NodeDaemonSet::Options so2;
        so2.daemon = dopt;
        so2.per_gpu = h->host->conf_bool("mapred.uda.daemon.per.gpu", true);
        const std::string cnt = h->host->get_conf("mapred.uda.daemon.count", "auto");
        so2.count = cnt == "auto" ? (so2.per_gpu ? std::max(1, uda::NodeDaemonSet::node_gpu_count()) : 1)
                                  : std::max(1, std::atoi(cnt.c_str()));
        std::string svc = h->host->get_conf("mapred.uda.gpu.merge.service", "auto");
        if (svc == "auto") svc = uda::MergeService::default_path(h->supplier->port());
        if (svc == "off" || svc == "0" || svc == "false") svc.clear();
        so2.service_path = svc;
        h->daemon = std::make_shared<uda::NodeDaemonSet>(so2, h->host.get());
        h->supplier->set_store(h->daemon);
      }
    }
  } catch (const std::exception& e) {
    UDA_LOG(uda::kError, "startNative failed: %s", e.what());
    return nullptr;
  }
  return h.release();
}

int uda_do_command(uda_handle* h, const char* cmd) {
  if (!h) return -1;
  std::lock_guard<std::mutex> g(h->mu);
  uda::HadoopCmd c;
  if (!uda::parse_cmd(cmd ? cmd : "", &c)) return fail_call(h, "C++ could not parse Hadoop command");
  try {
    if (h->is_merger) {
      if (h->remote) {
        try {
          h->remote->handle(cmd);
          return 0;
        } catch (const std::exception& e) {
          // the service runs this task for another user and refuses its files (local dirs outside the
          // node's own): this process merges instead, with the files its own user may touch
          if (c.header != uda::kInitMsg || std::string(e.what()).find("confined task") == std::string::npos) throw;
          UDA_LOG(uda::kWarn, "merge service refused the task's files (%s): merging in this process", e.what());
          h->remote->exit();
          h->remote.reset();
          h->task = std::make_unique<uda::ReduceTask>(h->opt, h->host.get());
        }
      }
      if (!h->task) return fail_call(h, "reduce task already closed");
      h->task->handle(c);
    } else {
      // mof_downcall_handler (MOFSupplierMain.cc:37-81): EXIT stops the supplier; JOB_OVER (sent by
      // the provider plugin when an application ends) releases the job's MOFs from the HBM store
      if (c.header == uda::kExitMsg && h->supplier) {
        h->service.reset();
        h->supplier->stop();
        h->daemon.reset();  // after the supplier: no worker asks it any more
        UDA_LOG(uda::kInfo, "MOFSupplier stopped");
      } else if (c.header == uda::kJobOverMsg && h->supplier && !c.params.empty()) {
        h->supplier->job_over(c.params[0]);
      }
    }
  } catch (const std::exception& e) {
    return fail_call(h, e.what());
  }
  return 0;
}

int uda_reduce_exit(uda_handle* h) {
  if (!h) return -1;
  std::lock_guard<std::mutex> g(h->mu);
  try {
    if (h->task) {
      h->task->exit();
      UDA_LOG(uda::kInfo, "reduce task closed: %s", h->task->stats_json().c_str());
    }
    if (h->remote) h->remote->exit();
    h->service.reset();
    if (h->supplier) h->supplier->stop();
    h->daemon.reset();
  } catch (const std::exception& e) {
    return fail_call(h, e.what());
  }
  return 0;
}

void uda_destroy(uda_handle* h) {
  if (!h) return;
  {
    std::lock_guard<std::mutex> g(h->mu);
    if (h->task) h->task->exit();
    if (h->remote) h->remote->exit();
    h->service.reset();
    if (h->supplier) h->supplier->stop();
    h->daemon.reset();
    h->task.reset();
    h->remote.reset();
    h->supplier.reset();
  }
  delete h;
}

const char* uda_last_error(uda_handle* h) { return h ? h->last_error.c_str() : ""; }

int uda_provider_register_mof(uda_handle* h, const char* job_id, const char* map_id, const void* data, int64_t len,
                              const int64_t* index, int32_t num_partitions) {
  return uda_provider_register_mof_device(h, job_id, map_id, data, len, index, num_partitions, -1);
}

int uda_provider_register_mof_device(uda_handle* h, const char* job_id, const char* map_id, const void* data,
                                     int64_t len, const int64_t* index, int32_t num_partitions, int32_t device) {
  if (!h || !h->supplier) return -1;
  std::vector<uda::IndexRec> recs((size_t)num_partitions);
  for (int i = 0; i < num_partitions; ++i) {
    recs[i].start_offset = index[3 * i];
    recs[i].raw_length = index[3 * i + 1];
    recs[i].part_length = index[3 * i + 2];
    recs[i].path = std::string(device >= 0 ? "hbm:" : "mem:") + job_id + "/" + map_id;
  }
  try {
    h->supplier->register_mof(job_id, map_id, (const uint8_t*)data, len, std::move(recs), device);
  } catch (const std::exception& e) {
    return fail_call(h, e.what());
  }
  return 0;
}

int uda_stats_json(uda_handle* h, char* out, int32_t outlen) {
  if (!h || !out || outlen <= 0) return -1;
  std::string s;
  if (h->task) {
    s = h->task->stats_json();
  } else if (h->remote) {
    s = h->remote->stats_json();
  } else if (h->supplier) {
    s = "{\"role\":\"mof_supplier\",\"requests\":" + std::to_string(h->supplier->requests()) +
        ",\"bytes_served\":" + std::to_string(h->supplier->bytes_served()) +
        ",\"descriptors_served\":" + std::to_string(h->supplier->descriptors_served()) +
        ",\"first_descriptor_request_boot_ms\":" + std::to_string(h->supplier->first_descriptor_request_boot_ms()) +
        ",\"port\":" +
        std::to_string(h->supplier->port()) + ",\"io\":\"" + h->supplier->io_backend() + "\",\"hbm_store\":" +
        h->supplier->hbm_stats_json() + "}";
  } else {
    s = "{}";
  }
  const int32_t n = (int32_t)std::min<size_t>(s.size(), (size_t)outlen - 1);
  std::memcpy(out, s.data(), (size_t)n);
  out[n] = 0;
  return (int)std::min<size_t>(s.size(), (size_t)INT32_MAX);  // the whole length: the caller may retry larger
}

}  // extern "C"
