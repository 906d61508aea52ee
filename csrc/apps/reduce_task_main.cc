// uda_reduce_task: one reduce task in a process of its own, the way Hadoop runs every reduce task (a
// YarnChild / TaskTracker child JVM that loads libuda.so, calls startNative as a NetMerger, sends INIT
// and one FETCH per map through doCommand, and reads the merged stream in dataFromUda).
//
// Reference: UdaBridge startNative / doCommandNative (src/UdaBridge.cc:187-295) and the NetMerger
// main (src/Merger/NetMergerMain.cc:44-77); the Java side's KVBuf copy + record walk of every
// delivered buffer (plugins/shared/.../UdaPlugin.java:369-402, 456-538) is the J2C consumer here.
//
//   uda_reduce_task [-D key=value]... [--kv-buf BYTES] [--expect RECORDS] [--check-order] -- <startNative args>
//
// stdin: one command string per line (INIT, FETCH..., optionally FINAL), sent to uda_do_command as
// they arrive; the task runs until its merged stream's EOF marker has been walked. stdout: one JSON
// line (consumer counts, the phases of the process's life, the task's own stats). Exit code 0 only if
// the task delivered every expected record with intact framing (and key order, --check-order).
// The consumer runs as the plugin does: dataFromUda copies into the KVBuf on the delivering thread, the
// walk runs on a walker thread of its own (the reducer's thread in the plugin), both pinned to the
// copier's last-level cache (j2c_sink.h). UDA_J2C_THREADS=0: both inline on the delivering thread.
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "uda/log.h"
#include "j2c_sink.h"
#include "uda/node_registry.h"
#include "uda/uda_bridge.h"
#include "uda/fd_table.h"

namespace {

double boot_ms() {  // CLOCK_BOOTTIME: the clock /proc/<pid>/stat start times count from
  timespec ts;
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

struct Host {
  std::map<std::string, std::string> conf;
  uda::gpu::J2CSink* sink = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  bool eof = false;
  std::string failure;
  double t_first_data = 0;
};

int data_cb(void* ctx, const void* buf, int32_t len) {
  auto* h = static_cast<Host*>(ctx);
  if (h->t_first_data == 0) h->t_first_data = boot_ms();
  return h->sink->consume(0, static_cast<const uint8_t*>(buf), len);
}
int conf_cb(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
  auto* h = static_cast<Host*>(ctx);
  std::string v = dflt ? dflt : "";
  auto it = h->conf.find(key);
  if (it != h->conf.end()) v = it->second;
  const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)outlen - 1);
  std::memcpy(out, v.data(), (size_t)n);
  out[n] = 0;
  return n;
}
void failure_cb(void* ctx, const char* reason) {
  auto* h = static_cast<Host*>(ctx);
  std::lock_guard<std::mutex> g(h->mu);
  if (h->failure.empty()) h->failure = reason && *reason ? reason : "failure";
  h->cv.notify_all();
}
void log_cb(void*, const char* msg, int32_t sev) {
  if (sev <= 2) std::fprintf(stderr, "[uda_reduce_task %d] %s\n", (int)getpid(), msg);
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if ((unsigned char)c < 0x20) {
      o += ' ';
      continue;
    }
    o += c;
  }
  return o;
}

}  // namespace

int main(int argc, char** argv) {
  const double t_main = boot_ms();
  uda::pregrow_fd_table(1 << 14);  // delivery rings (memfds), fetch connections
  uda::install_crash_reporter("uda_reduce_task");
  const double t_exec = (double)uda::process_start_ticks((int)getpid()) * 1000.0 / (double)sysconf(_SC_CLK_TCK);
  Host host;
  int64_t kv_buf = 1 << 20, expect = -1;
  bool kv_buf_set = false;
  bool check_order = false;
  std::vector<std::string> start_args;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-D" && i + 1 < argc) {
      const std::string kv = argv[++i];
      const size_t eq = kv.find('=');
      if (eq != std::string::npos) host.conf[kv.substr(0, eq)] = kv.substr(eq + 1);
    } else if (a == "--kv-buf" && i + 1 < argc) {
      kv_buf = std::atoll(argv[++i]);
      kv_buf_set = true;
    } else if (a == "--expect" && i + 1 < argc) {
      expect = std::atoll(argv[++i]);
    } else if (a == "--check-order") {
      check_order = true;
    } else if (a == "--") {
      for (++i; i < argc; ++i) start_args.push_back(argv[i]);
    } else {
      std::fprintf(stderr, "usage: %s [-D key=value]... [--kv-buf B] [--expect N] [--check-order] -- <args>\n", argv[0]);
      return 2;
    }
  }
  // the job's configuration holds only the -D keys (a node-shape run passes none); --kv-buf sets the
  // dataFromUda buffer size on both sides
  if (kv_buf_set) host.conf["mapred.uda.kv.buf.size"] = std::to_string(kv_buf);
  // the plugin's two threads unless UDA_J2C_THREADS=0: a service-hosted cold task 12.8-13.4 GB/s in 5 of 5
  // trials against 10.7-11.3 inline (profiles/r5_j2c_consumer_ab.md)
  uda::gpu::J2CSink sink(1, kv_buf, uda::gpu::J2CSink::plugin_threaded());
  sink.set_check_order(check_order);
  sink.set_key_kind(1);
  sink.set_on_eof([&host](int) {
    std::lock_guard<std::mutex> g(host.mu);
    host.eof = true;
    host.cv.notify_all();
  });
  host.sink = &sink;
  uda_callbacks cb{};
  cb.ctx = &host;
  cb.data_from_uda = data_cb;
  cb.get_conf = conf_cb;
  cb.failure = failure_cb;
  cb.log = log_cb;
  std::vector<const char*> av;
  for (auto& s : start_args) av.push_back(s.c_str());
  uda_handle* h = uda_start(1, (int)av.size(), av.data(), 2, 0, &cb);
  const double t_started = boot_ms();
  if (!h) {
    std::printf("{\"error\":\"uda_start failed\"}\n");
    return 1;
  }
  double t_init = 0, t_first_fetch = 0, t_last_cmd = 0;
  std::string err;
  for (std::string line; std::getline(std::cin, line);) {
    if (line.empty()) continue;
    const size_t c = line.find(':');  // "<count>:<id>:...": FETCH is id 4 (uda/cmd.h)
    const bool fetch = c != std::string::npos && line.compare(c + 1, 2, "4:") == 0;
    if (fetch && t_first_fetch == 0) t_first_fetch = boot_ms();
    if (uda_do_command(h, line.c_str()) != 0) {
      err = uda_last_error(h);
      break;
    }
    if (t_init == 0) t_init = boot_ms();
    t_last_cmd = boot_ms();
  }
  {
    std::unique_lock<std::mutex> lk(host.mu);
    if (err.empty() && !host.cv.wait_for(lk, std::chrono::seconds(900), [&] { return host.eof || !host.failure.empty(); }))
      err = "no EOF within 900 s";
    if (err.empty() && !host.failure.empty()) err = host.failure;
  }
  const double t_eof = boot_ms();
  (void)uda_reduce_exit(h);
  const std::string js = uda_stats_string(h);  // any size (free-text fields can make it long)
  uda_destroy(h);
  sink.flush();
  const double t_end = boot_ms();
  if (err.empty() && sink.error(0) != 0) err = "consumer framing error " + std::to_string(sink.error(0));
  if (err.empty() && expect >= 0 && sink.records(0) != expect)
    err = "consumer parsed " + std::to_string(sink.records(0)) + " records, expected " + std::to_string(expect);
  if (err.empty() && check_order && sink.order_errors(0) != 0)
    err = std::to_string(sink.order_errors(0)) + " records out of order";
  std::printf(
      "{\"pid\":%d,\"records\":%lld,\"bytes\":%lld,\"buffers\":%lld,\"order_errors\":%lld,\"error\":\"%s\","
      "\"exec_to_main_ms\":%.1f,\"start_ms\":%.1f,\"init_ms\":%.1f,\"first_fetch_ms\":%.1f,\"fetch_to_first_data_ms\":%.1f,"
      "\"fetch_to_eof_ms\":%.1f,\"exit_ms\":%.1f,\"exec_to_end_ms\":%.1f,\"t_exec_boot_ms\":%.1f,\"t_end_boot_ms\":%.1f,"
      "\"j2c\":%s,\"task\":%s}\n",
      (int)getpid(), (long long)sink.records(0), (long long)sink.bytes(0), (long long)sink.buffers(0),
      (long long)sink.order_errors(0), json_escape(err).c_str(), t_main - t_exec, t_started - t_main,
      t_init > 0 ? t_init - t_started : -1.0, t_first_fetch > 0 ? t_first_fetch - t_exec : -1.0,
      t_first_fetch > 0 && host.t_first_data > 0 ? host.t_first_data - t_first_fetch : -1.0,
      t_first_fetch > 0 ? t_eof - t_first_fetch : -1.0, t_end - t_eof, t_end - t_exec, t_exec, t_end, sink.placement_json(0).c_str(), js.c_str());
  std::fflush(stdout);
  (void)t_last_cmd;
  return err.empty() ? 0 : 1;
}
