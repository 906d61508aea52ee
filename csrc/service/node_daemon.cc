// The node daemon and its supervisor in the provider front end. See node_daemon.h.
#include "node_daemon.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <signal.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <poll.h>
#include <thread>

#include "../consumer/reduce_task.h"
#include "../gpu/device_ptr.h"
#include "../gpu/hbm_ledger.h"
#include "merge_service.h"
#include "uda/cmd.h"
#include "uda/error.h"
#include "uda/frame.h"
#include "uda/log.h"
#include "uda/stall_probe.h"
#include "uda/start_trace.h"
#include "uda/topology.h"
#include "uda/transport.h"
#include "uda/uda_bridge.h"
#include "uda/thread_name.h"

extern char** environ;

namespace uda {

namespace {

using frame::get;
using frame::get_str;
using frame::put;
using frame::put_str;
using frame::recv_msg;
using frame::send_msg;

enum DMsg : uint32_t {
  // front end -> daemon
  kDStart = 1,          // str startNative args ('\0'-joined), i32 data port
  kDAcquire = 2,        // u64 id, str job, str path, str holder, i64 offset, i64 len
  kDRelease = 3,        // str path, str holder
  kDReleaseHolder = 4,  // str job, str holder
  kDJobOver = 5,        // str job
  kDStats = 6,          // u64 id
  kDExit = 7,
  kDConfReply = 8,  // u32 id, str value
  kDAdopt = 9,      // + fd: a merge-service client connection the front end's router accepted
  // daemon -> front end
  kDReady = 20,       // str merge service path ("" = none), i64 store bytes
  kDFailed = 21,      // str why
  kDAcquired = 22,    // u64 id, i32 status, str descriptor or why
  kDConfReq = 23,     // u32 id, str key, str default
  kDLog = 24,         // i32 severity, str message
  kDStatsReply = 25,  // u64 id, str json
  kDSessionEnd = 26,  // u64 HELLO token: a routed merge-service session is over (or was refused)
};

std::string join_args(const std::vector<std::string>& a) {
  std::string s;
  for (size_t i = 0; i < a.size(); ++i) {
    if (i) s.push_back('\0');
    s += a[i];
  }
  return s;
}

std::vector<std::string> split_args(const std::string& s) {
  std::vector<std::string> v;
  if (s.empty()) return v;
  for (size_t b = 0; b <= s.size();) {
    const size_t e = s.find('\0', b);
    v.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) break;
    b = e + 1;
  }
  return v;
}

// "a, b,c" -> {"a", "b", "c"} (configuration lists)
std::vector<std::string> split_list(const std::string& s) {
  std::vector<std::string> v;
  for (size_t b = 0; b <= s.size();) {
    size_t e = s.find(',', b);
    if (e == std::string::npos) e = s.size();
    std::string t = s.substr(b, e - b);
    while (!t.empty() && t.front() == ' ') t.erase(0, 1);
    while (!t.empty() && t.back() == ' ') t.pop_back();
    if (!t.empty()) v.push_back(t);
    b = e + 1;
  }
  return v;
}

std::string exit_text(int status) {
  if (WIFEXITED(status)) return "exit code " + std::to_string(WEXITSTATUS(status));
  if (WIFSIGNALED(status)) return std::string("signal ") + strsignal(WTERMSIG(status));
  return "status " + std::to_string(status);
}

// wait for `pid` up to `s` seconds, then SIGKILL it; returns how it ended
std::string reap(pid_t pid, double s) {
  int status = 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const pid_t r = ::waitpid(pid, &status, WNOHANG);
    if (r == pid) return exit_text(status);
    if (r < 0) return errno == ECHILD ? "already reaped" : std::string("waitpid: ") + strerror(errno);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::duration<double>(s)) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  ::kill(pid, SIGKILL);
  if (::waitpid(pid, &status, 0) == pid) return "killed after " + std::to_string((int)s) + " s (" + exit_text(status) + ")";
  return "killed";
}

}  // namespace

// ==================================================================================== front end side

std::string NodeDaemonClient::default_exe() {
  if (const char* e = std::getenv("UDA_DAEMON_EXE")) return e;
  Dl_info info{};
  if (!dladdr(reinterpret_cast<void*>(&uda_start), &info) || !info.dli_fname) return "";
  std::string dir = info.dli_fname;
  const size_t slash = dir.rfind('/');
  dir = slash == std::string::npos ? std::string(".") : dir.substr(0, slash);
  for (const std::string& c : {dir + "/../bin/uda_mof_supplier", dir + "/bin/uda_mof_supplier", dir + "/uda_mof_supplier"})
    if (::access(c.c_str(), X_OK) == 0) return c;
  return "";
}

bool NodeDaemonClient::node_has_gpu() { return ::access("/dev/kfd", R_OK | W_OK) == 0; }

NodeDaemonClient::NodeDaemonClient(const Options& o, Host* host) : opt_(o), host_(host) {
  if (opt_.exe.empty()) opt_.exe = default_exe();
  if (opt_.exe.empty()) {
    why_ = "node daemon executable (uda_mof_supplier) not found next to libuda.so";
    UDA_LOG(kWarn, "%s: descriptor fetches are declined (reducers fetch bytes)", why_.c_str());
    return;
  }
  if (!spawn()) return;
  wait_ready(opt_.start_timeout_s);
  std::lock_guard<std::mutex> g(mu_);
  if (ready_)
    UDA_LOG(kInfo, "node daemon pid %d ready: HBM store %.1f GB, merge service %s", (int)pid_.load(),
            (double)store_bytes_ / 1e9, service_path_.empty() ? "off" : service_path_.c_str());
  else
    UDA_LOG(kWarn, "node daemon not ready (%s): descriptor fetches are declined (reducers fetch bytes)", why_.c_str());
}

NodeDaemonClient::~NodeDaemonClient() {
  {
    // under mu_: a restart on a reader thread (daemon_gone -> spawn) checks it under the same lock, so
    // no daemon is started (and no reader_ replaced) from here on
    std::lock_guard<std::mutex> g(mu_);
    stopping_ = true;
    cv_.notify_all();
  }
  send(kDExit, "");
  const pid_t p = pid_.exchange(0);
  if (p > 0) {
    const std::string how = reap(p, 30);
    UDA_LOG(kInfo, "node daemon pid %d stopped (%s)", (int)p, how.c_str());
  }
  std::vector<std::thread> readers;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);  // the reader sees EOF
    if (reader_.joinable()) readers.push_back(std::move(reader_));
    for (auto& t : old_readers_)
      if (t.joinable()) readers.push_back(std::move(t));
    old_readers_.clear();
  }
  for (auto& t : readers) t.join();
  // a daemon a restart published before it saw stopping_ (between the exchange above and now)
  const pid_t late = pid_.exchange(0);
  if (late > 0) {
    ::kill(late, SIGKILL);
    UDA_LOG(kInfo, "node daemon pid %d (late restart) stopped (%s)", (int)late, reap(late, 5).c_str());
  }
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
}

bool NodeDaemonClient::spawn() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stopping_) return false;
  }
  int sv[2];
  if (::socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) {
    std::lock_guard<std::mutex> g(mu_);
    why_ = std::string("socketpair: ") + strerror(errno);
    return false;
  }
  // the daemon's end lands on a fixed descriptor number in the child (dup2 there clears close-on-exec)
  const int child_fd = sv[1] == 100 ? 101 : 100;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, sv[1], child_fd);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  std::string log = opt_.log_path.empty() ? std::string("/dev/null") : opt_.log_path;
  if (const int probe = ::open(log.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644); probe >= 0) {
    ::close(probe);
  } else {
    log = "/dev/null";  // an unwritable log must not keep the daemon from starting
  }
  posix_spawn_file_actions_addopen(&fa, 1, log.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  posix_spawn_file_actions_adddup2(&fa, 1, 2);
  posix_spawnattr_t attr;
  posix_spawnattr_init(&attr);
  sigset_t none, all;
  sigemptyset(&none);
  sigfillset(&all);
  posix_spawnattr_setsigmask(&attr, &none);    // a JVM host blocks signals the daemon must see
  posix_spawnattr_setsigdefault(&attr, &all);  // and installs handlers it must not inherit
  posix_spawnattr_setflags(&attr, POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF);
  const std::string fd_arg = std::to_string(child_fd);
  std::vector<char*> argv = {const_cast<char*>(opt_.exe.c_str()), const_cast<char*>("--daemon-fd"),
                             const_cast<char*>(fd_arg.c_str()), nullptr};
  // The daemon starts a wave of hosted tasks at once (a dozen threads each); every thread stack mmap, every
  // new malloc arena and each of its growth steps takes the address-space lock for writing, and in that
  // convoy the control channel's own allocations waited 100-250 ms (UDA_STALL_PROBE). So the daemon keeps
  // exited threads' stacks (1 GiB cache, virtual), uses at most 8 arenas made writable whole at creation
  // (64 MiB top pad), never trims them, and serves blocks under 32 MiB from them rather than from mmap.
  // UDA_DAEMON_TUNABLES replaces the set ("" for glibc's defaults).
  const char* tun_env = std::getenv("UDA_DAEMON_TUNABLES");
  const std::string tun = tun_env ? tun_env
                                  : "glibc.pthread.stack_cache_size=1073741824:glibc.malloc.arena_max=8:"
                                    "glibc.malloc.top_pad=67108864:glibc.malloc.trim_threshold=268435456:"
                                    "glibc.malloc.mmap_threshold=33554432";
  std::vector<std::string> env_store;
  bool had_tunables = false;
  for (char** e = environ; e && *e; ++e) {
    std::string kv = *e;
    if (kv.rfind("GLIBC_TUNABLES=", 0) == 0) {
      had_tunables = true;
      if (!tun.empty()) kv += ":" + tun;  // the later setting of a tunable wins
    }
    env_store.push_back(std::move(kv));
  }
  if (!had_tunables && !tun.empty()) env_store.push_back("GLIBC_TUNABLES=" + tun);
  std::vector<char*> envp;
  for (auto& kv : env_store) envp.push_back(const_cast<char*>(kv.c_str()));
  envp.push_back(nullptr);
  pid_t pid = 0;
  const int rc = ::posix_spawn(&pid, opt_.exe.c_str(), &fa, &attr, argv.data(), envp.data());
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&attr);
  ::close(sv[1]);
  if (rc != 0) {
    ::close(sv[0]);
    std::lock_guard<std::mutex> g(mu_);
    why_ = "cannot start " + opt_.exe + ": " + strerror(rc);
    UDA_LOG(kError, "%s", why_.c_str());
    return false;
  }
  uint64_t gen;
  {
    std::lock_guard<std::mutex> gs(send_mu_);  // lock order: send_mu_, then mu_ (as in send())
    std::unique_lock<std::mutex> g(mu_);
    if (stopping_) {  // the client is being destroyed: this daemon never serves
      g.unlock();
      ::close(sv[0]);
      ::kill(pid, SIGKILL);
      (void)reap(pid, 5);
      return false;
    }
    if (fd_ >= 0) ::close(fd_);
    fd_ = sv[0];
    gen = ++gen_;
    failed_start_ = false;
    why_ = "node daemon starting";
    pid_ = pid;
    if (reader_.joinable()) old_readers_.push_back(std::move(reader_));  // maybe this very thread (a restart)
    reader_ = std::thread([this, fd = sv[0], gen] { reader_main(fd, gen); });
  }
  std::string st;
  put_str(st, join_args(opt_.start_args));
  put<int32_t>(st, opt_.data_port);
  put<int32_t>(st, opt_.device);
  put<int32_t>(st, opt_.ndaemons);
  send(kDStart, st);
  UDA_LOG(kInfo, "node daemon %s started, pid %d (generation %llu)", opt_.exe.c_str(), (int)pid,
          (unsigned long long)gen);
  return true;
}

bool NodeDaemonClient::wait_ready(double s) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait_for(lk, std::chrono::duration<double>(s), [&] { return ready_.load() || failed_start_ || stopping_; });
  if (!ready_ && !failed_start_ && pid_.load() > 0 && why_ == "node daemon starting")
    why_ = "node daemon not ready within " + std::to_string((int)s) + " s";
  return ready_;
}

std::string NodeDaemonClient::why() const {
  std::lock_guard<std::mutex> g(mu_);
  return why_;
}

std::string NodeDaemonClient::service_path() const {
  std::lock_guard<std::mutex> g(mu_);
  return service_path_;
}

bool NodeDaemonClient::send(uint32_t type, const std::string& payload) {
  std::lock_guard<std::mutex> gs(send_mu_);
  int fd;
  {
    std::lock_guard<std::mutex> g(mu_);
    fd = fd_;
  }
  return fd >= 0 && send_msg(fd, type, payload);
}

void NodeDaemonClient::reader_main(int fd, uint64_t gen) {
  for (;;) {
    uint32_t t;
    std::string p;
    int pfd;
    if (!recv_msg(fd, &t, &p, &pfd)) break;
    if (pfd >= 0) ::close(pfd);
    if (t == kDAcquired) {
      const uint64_t id = get<uint64_t>(p, 0);
      const int32_t status = get<int32_t>(p, 8);
      size_t at = 12;
      const std::string desc = get_str(p, &at);
      Done done;
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = pending_.find(id);
        if (it == pending_.end()) continue;
        done = std::move(it->second);
        pending_.erase(it);
      }
      start_trace("fe_acquired", id);
      done(status, desc);
      start_trace("fe_acquired_done", id);
    } else if (t == kDConfReq) {
      const uint32_t id = get<uint32_t>(p, 0);
      size_t at = 4;
      const std::string key = get_str(p, &at), dflt = get_str(p, &at);
      std::string r;
      put<uint32_t>(r, id);
      put_str(r, host_ ? host_->get_conf(key, dflt) : dflt);
      std::lock_guard<std::mutex> gs(send_mu_);
      (void)send_msg(fd, kDConfReply, r);
    } else if (t == kDLog) {
      const int32_t sev = get<int32_t>(p, 0);
      size_t at = 4;
      const std::string msg = get_str(p, &at);
      UDA_LOG(sev, "[node daemon %d] %s", (int)pid_.load(), msg.c_str());
    } else if (t == kDReady) {
      size_t at = 0;
      const std::string svc = get_str(p, &at);
      const int64_t bytes = get<int64_t>(p, at);
      std::lock_guard<std::mutex> g(mu_);
      if (gen != gen_) continue;
      service_path_ = svc;
      store_bytes_ = bytes;
      why_.clear();
      ready_ = true;
      cv_.notify_all();
    } else if (t == kDFailed) {
      size_t at = 0;
      const std::string w = get_str(p, &at);
      std::lock_guard<std::mutex> g(mu_);
      if (gen != gen_) continue;
      why_ = w;
      failed_start_ = true;
      cv_.notify_all();
    } else if (t == kDStatsReply) {
      const uint64_t id = get<uint64_t>(p, 0);
      size_t at = 8;
      std::lock_guard<std::mutex> g(mu_);
      stats_replies_[id] = get_str(p, &at);
      cv_.notify_all();
    } else if (t == kDSessionEnd) {
      std::lock_guard<std::mutex> g(mu_);
      if (gen == gen_) sessions_.erase(get<uint64_t>(p, 0));
    }
  }
  daemon_gone(gen, "control connection closed");
}

void NodeDaemonClient::daemon_gone(uint64_t gen, const std::string& why) {
  std::map<uint64_t, Done> pending;
  bool restart = false;
  std::string how;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (gen != gen_) return;
    ready_ = false;
    pending.swap(pending_);
    sessions_.clear();  // the hosted tasks of that moment are gone with it
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
  }
  const pid_t p = pid_.exchange(0);
  if (p > 0) how = reap(p, 5);
  {
    std::lock_guard<std::mutex> g(mu_);
    const bool was_started = !failed_start_;
    why_ = "node daemon" + (p > 0 ? " pid " + std::to_string((int)p) : std::string()) + " gone (" + why +
           (how.empty() ? "" : ", " + how) + ")";
    restart = !stopping_ && was_started && restarts_.load() < opt_.max_restarts;
    cv_.notify_all();
  }
  if (!stopping_) UDA_LOG(kError, "%s; %s", why_.c_str(), restart ? "restarting it" : "descriptor fetches are declined from now on");
  for (auto& kv : pending) kv.second(kNotDeviceResident, "node daemon gone: " + why);
  if (restart) {
    restarts_++;
    std::this_thread::sleep_for(std::chrono::seconds(1));
    if (!stopping_ && spawn()) wait_ready(opt_.start_timeout_s);
  }
}

bool NodeDaemonClient::acquire(const std::string& job, const std::string& path, const std::string& holder,
                               int64_t offset, int64_t len, Done done, std::string* why) {
  uint64_t id;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!ready_) {
      if (why) *why = why_;
      return false;
    }
    id = next_id_++;
    pending_[id] = std::move(done);
  }
  std::string m;
  put<uint64_t>(m, id);
  put_str(m, job);
  put_str(m, path);
  put_str(m, holder);
  put<int64_t>(m, offset);
  put<int64_t>(m, len);
  if (send(kDAcquire, m)) return true;
  std::lock_guard<std::mutex> g(mu_);
  if (pending_.erase(id) == 0) return true;  // the daemon-gone path already answered it
  if (why) *why = "node daemon unreachable";
  return false;
}

bool NodeDaemonClient::adopt(int fd, uint64_t token) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!ready_) return false;
    if (token) sessions_.insert(token);
  }
  std::lock_guard<std::mutex> gs(send_mu_);
  int cfd;
  {
    std::lock_guard<std::mutex> g(mu_);
    cfd = fd_;
  }
  if (cfd >= 0 && send_msg(cfd, kDAdopt, "", fd)) return true;
  std::lock_guard<std::mutex> g(mu_);
  if (token) sessions_.erase(token);
  return false;
}

int NodeDaemonClient::live_sessions() const {
  std::lock_guard<std::mutex> g(mu_);
  return (int)sessions_.size();
}

void NodeDaemonClient::release(const std::string& path, const std::string& holder) {
  if (!ready_) return;
  std::string m;
  put_str(m, path);
  put_str(m, holder);
  send(kDRelease, m);
}

void NodeDaemonClient::release_holder(const std::string& job, const std::string& holder) {
  if (!ready_) return;
  std::string m;
  put_str(m, job);
  put_str(m, holder);
  send(kDReleaseHolder, m);
}

void NodeDaemonClient::job_over(const std::string& job) {
  if (!ready_) return;
  std::string m;
  put_str(m, job);
  send(kDJobOver, m);
}

std::string NodeDaemonClient::stats_json() {
  std::string body = "{}";
  uint64_t id = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (ready_) id = next_id_++;
  }
  if (id) {
    std::string m;
    put<uint64_t>(m, id);
    if (send(kDStats, m)) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_for(lk, std::chrono::seconds(10), [&] { return stats_replies_.count(id) || !ready_; });
      auto it = stats_replies_.find(id);
      if (it != stats_replies_.end()) {
        body = it->second;
        stats_replies_.erase(it);
      }
    }
  }
  std::string d;
  {
    std::lock_guard<std::mutex> g(mu_);
    std::string w;
    for (char c : why_) w += (c == '"' || c == '\\') ? ' ' : c;
    d = "\"daemon\":{\"pid\":" + std::to_string((int)pid_.load()) + ",\"ready\":" + (ready_ ? "true" : "false") +
        ",\"restarts\":" + std::to_string(restarts_.load()) + ",\"service\":\"" + service_path_ + "\",\"why\":\"" + w +
        "\"}";
  }
  if (body.size() < 2 || body.back() != '}') body = "{}";
  return body.size() == 2 ? "{" + d + "}" : body.substr(0, body.size() - 1) + "," + d + "}";
}

// ==================================================================================== daemon side

namespace {

struct Daemon {
  int ctl = -1;
  std::mutex send_mu;
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint32_t, std::string> conf_replies;
  uint32_t next_conf = 1;
  bool closed = false, exit_req = false;
  std::shared_ptr<DeviceStore> store;
  std::unique_ptr<MergeService> svc;
  std::thread prewarm;  // GPU prewarm for the first wave of hosted tasks
  std::atomic<int> prewarm_tasks{0}, prewarm_done{0};
  std::atomic<int64_t> prewarm_us{0};
  std::deque<std::string> starts;

  bool send(uint32_t t, const std::string& p) {
    std::lock_guard<std::mutex> g(send_mu);
    return send_msg(ctl, t, p);
  }

  // getConfData of the NodeManager, through the front end
  std::string conf(const std::string& key, const std::string& dflt) {
    uint32_t id;
    {
      std::lock_guard<std::mutex> g(mu);
      if (closed) return dflt;
      id = next_conf++;
    }
    std::string m;
    put<uint32_t>(m, id);
    put_str(m, key);
    put_str(m, dflt);
    if (!send(kDConfReq, m)) return dflt;
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return closed || conf_replies.count(id); })) return dflt;
    auto it = conf_replies.find(id);
    if (it == conf_replies.end()) return dflt;
    std::string v = std::move(it->second);
    conf_replies.erase(it);
    return v;
  }

  static void log_sink(void* ctx, const char* msg, int sev) {
    auto* d = static_cast<Daemon*>(ctx);
    std::string m;
    put<int32_t>(m, sev);
    put_str(m, msg ? msg : "");
    (void)d->send(kDLog, m);
  }

  std::string stats() {
    std::shared_ptr<DeviceStore> st;
    std::string ms = "{}";
    {
      std::lock_guard<std::mutex> g(mu);
      st = store;
      if (svc) ms = svc->stats_json();
    }
    std::string s = st ? st->stats_json() : "{}";
    char pw[96];
    std::snprintf(pw, sizeof(pw), "\"prewarm\":{\"tasks\":%d,\"done\":%s,\"ms\":%.1f}", prewarm_tasks.load(),
                  prewarm_done.load() ? "true" : "false", (double)prewarm_us.load() / 1e3);
    ms = ms + "," + pw;
    // the allocator settings the front end spawned this daemon with (glibc's view, after its parsing)
    std::string tun = std::getenv("GLIBC_TUNABLES") ? std::getenv("GLIBC_TUNABLES") : "";
    for (char& c : tun)
      if (!std::isalnum((unsigned char)c) && !std::strchr("._=:", c)) c = '_';  // JSON-safe
    ms += ",\"glibc_tunables\":\"" + tun + "\"";
    return s.size() <= 2 ? "{\"merge_service\":" + ms + "}" : s.substr(0, s.size() - 1) + ",\"merge_service\":" + ms + "}";
  }

  void read_loop() {
    name_thread("uda-daemon-ctl");
    stall_probe_watch();
    for (;;) {
      uint32_t t;
      std::string p;
      int pfd;
      if (!recv_msg(ctl, &t, &p, &pfd)) break;
      if (t == kDAdopt) {  // a client connection routed to this daemon's merge service
        start_trace("daemon_adopt", 0);
        std::lock_guard<std::mutex> g(mu);
        if (svc && pfd >= 0)
          svc->adopt(pfd);
        else if (pfd >= 0)
          ::close(pfd);
        continue;
      }
      if (pfd >= 0) ::close(pfd);
      start_trace(t == kDAcquire ? "daemon_acquire_msg" : "daemon_msg", t);
      std::shared_ptr<DeviceStore> st;
      {
        std::lock_guard<std::mutex> g(mu);
        st = store;
      }
      if (t == kDConfReply) {
        size_t at = 4;
        std::lock_guard<std::mutex> g(mu);
        conf_replies[get<uint32_t>(p, 0)] = get_str(p, &at);
        cv.notify_all();
      } else if (t == kDStart) {
        std::lock_guard<std::mutex> g(mu);
        starts.push_back(p);
        cv.notify_all();
      } else if (t == kDAcquire) {
        const uint64_t id = get<uint64_t>(p, 0);
        size_t at = 8;
        const std::string job = get_str(p, &at), path = get_str(p, &at), holder = get_str(p, &at);
        const int64_t off = get<int64_t>(p, at), len = get<int64_t>(p, at + 8);
        auto reply = [this, id](int status, const std::string& desc) {
          std::string r;
          put<uint64_t>(r, id);
          put<int32_t>(r, status);
          put_str(r, desc);
          start_trace("daemon_reply", id);
          (void)send(kDAcquired, r);
          start_trace("daemon_reply_sent", id);
        };
        std::string why;
        if (!st) {
          reply(kNotDeviceResident, "the node daemon has no HBM store");
        } else if (!st->acquire(job, path, holder, off, len, reply, &why)) {
          reply(kNotDeviceResident, "provider HBM store: " + why);
        }
        start_trace("daemon_acquire_done", id);
      } else if (t == kDRelease) {
        size_t at = 0;
        const std::string path = get_str(p, &at), holder = get_str(p, &at);
        if (st) st->release(path, holder);
      } else if (t == kDReleaseHolder) {
        size_t at = 0;
        const std::string job = get_str(p, &at), holder = get_str(p, &at);
        if (st) st->release_holder(job, holder);
      } else if (t == kDJobOver) {
        size_t at = 0;
        if (st) st->job_over(get_str(p, &at));
      } else if (t == kDStats) {
        std::string r;
        put<uint64_t>(r, get<uint64_t>(p, 0));
        put_str(r, stats());
        (void)send(kDStatsReply, r);
      } else if (t == kDExit) {
        std::lock_guard<std::mutex> g(mu);
        exit_req = true;
        cv.notify_all();
      }
    }
    std::lock_guard<std::mutex> g(mu);
    closed = true;
    cv.notify_all();
  }
};

// "auto" / bytes (> 1) / a fraction of the device's HBM budget (0 < f <= 1) of every store device
int64_t store_capacity(const std::string& conf, const std::vector<int>& devices) {
  double f = 0.6;  // auto: the rest of the budget stays with the hosted tasks' working sets
  if (conf != "auto") {
    const double v = std::atof(conf.c_str());
    if (v > 1.0) return (int64_t)v;
    if (v <= 0) return 0;
    f = v;
  }
  int64_t total = 0;
  for (int d : devices) total += (int64_t)((double)gpu::HbmLedger::get().budget(d) * f);
  return total;
}

}  // namespace

int run_node_daemon(int ctl_fd) {
  ::signal(SIGPIPE, SIG_IGN);
  auto d = std::make_unique<Daemon>();
  d->ctl = ctl_fd;
  std::thread reader([&] { d->read_loop(); });
  int rc = 0;
  try {
    // START comes first: the provider's startNative arguments and its TCP port
    std::string start;
    {
      std::unique_lock<std::mutex> lk(d->mu);
      d->cv.wait(lk, [&] { return d->closed || !d->starts.empty(); });
      if (d->starts.empty()) throw UdaError("front end gone before START");
      start = d->starts.front();
    }
    size_t at = 0;
    const std::vector<std::string> args = split_args(get_str(start, &at));
    const int port = get<int32_t>(start, at);
    // a per-GPU daemon (node_daemon.h NodeDaemonSet): its GPU, how many daemons the node runs, and the
    // merge service without a listener of its own (the front end routes client connections to it)
    const int my_device = start.size() >= at + 8 ? get<int32_t>(start, at + 4) : -1;
    const int ndaemons = start.size() >= at + 12 ? std::max(1, get<int32_t>(start, at + 8)) : 1;
    NetlevOptions opt;
    std::string err;
    if (!parse_options(args, &opt, &err)) throw UdaError("bad startNative options: " + err);
    log_set_sink(&Daemon::log_sink, d.get());  // the daemon's log lands in the NodeManager's
    log_set_threshold((int)std::atoi(d->conf("mapred.uda.log.level", std::to_string(log_threshold())).c_str()));
    UDA_LOG(kInfo, "node daemon up (pid %d), provider port %d", (int)getpid(), port);
    // GPUs: every visible one carries a share of the store; tasks are placed over all of them
    const std::vector<std::string> keys = gpu::visible_device_keys();
    const std::string force = d->conf("mapred.uda.daemon", "auto");
    if (keys.empty() && force != "1" && force != "true")
      throw UdaError("no HIP device visible to the node daemon");
    const double budget = std::atof(d->conf("mapred.uda.gpu.hbm.budget", "0").c_str());
    std::vector<int> devs;
    std::string dconf = d->conf("mapred.uda.provider.hbm.devices", "all");
    if (my_device >= 0) {
      if (!keys.empty() && my_device >= (int)keys.size())
        throw UdaError("node daemon for GPU " + std::to_string(my_device) + " but " + std::to_string(keys.size()) +
                       " GPU(s) are visible");
      if (!keys.empty()) devs.push_back(my_device);
    } else if (dconf == "all") {
      for (int i = 0; i < (int)keys.size(); ++i) devs.push_back(i);
    } else {
      for (size_t b = 0; b <= dconf.size();) {
        const size_t e = dconf.find(',', b);
        const std::string t = dconf.substr(b, e == std::string::npos ? std::string::npos : e - b);
        if (!t.empty()) devs.push_back(std::atoi(t.c_str()));
        if (e == std::string::npos) break;
        b = e + 1;
      }
    }
    for (int dv : devs) gpu::HbmLedger::get().configure(dv, budget);
    int64_t store_bytes = 0;
    if (!keys.empty() && !devs.empty()) {
      LocalStoreOptions so;
      so.devices = devs;
      so.capacity = store_capacity(d->conf("mapred.uda.provider.hbm.bytes", "auto"), devs);
      so.lease_s = std::atof(d->conf("mapred.uda.provider.hbm.lease.s", "600").c_str());
      so.idle_evict_s = std::atof(d->conf("mapred.uda.provider.hbm.idle.evict.s", "30").c_str());
      so.cached_read = std::atoi(d->conf("mapred.uda.provider.hbm.cached.read", "1").c_str()) != 0;
      if (so.capacity > 0) {
        std::lock_guard<std::mutex> g(d->mu);
        d->store = make_local_device_store(so);
        store_bytes = so.capacity;
      }
    }
    // the merge service, after which pinned host memory of this process is shareable with its clients
    std::string svc_path = d->conf("mapred.uda.gpu.merge.service", "auto");
    if (svc_path == "auto") svc_path = MergeService::default_path(port);
    if (svc_path == "off" || svc_path == "0" || svc_path == "false") svc_path.clear();
    if (!svc_path.empty()) {
      MergeService::Options mo;
      mo.path = my_device >= 0 ? std::string() : svc_path;  // per-GPU: the front end listens and routes
      if (my_device >= 0) {
        mo.force_device = my_device;
        Daemon* dp = d.get();
        mo.session_closed = [dp](uint64_t token) {
          std::string m;
          put<uint64_t>(m, token);
          (void)dp->send(kDSessionEnd, m);
        };
      }
      mo.users = d->conf("mapred.uda.gpu.merge.service.users", "");
      mo.max_sessions = (int)std::atoi(d->conf("mapred.uda.gpu.merge.service.max.sessions", "256").c_str());
      mo.max_sessions_per_user =
          (int)std::atoi(d->conf("mapred.uda.gpu.merge.service.max.sessions.per.user", "64").c_str());
      // where a foreign user's hosted task may keep files: the node's own local directories
      std::string roots = d->conf("mapred.uda.gpu.merge.service.local.dirs", "");
      if (roots.empty()) roots = d->conf("yarn.nodemanager.local-dirs", "");
      if (roots.empty()) roots = d->conf("mapred.local.dir", "");
      for (const std::string& r : split_list(roots)) {
        char buf[PATH_MAX];
        if (::realpath(r.c_str(), buf)) mo.local_roots.emplace_back(buf);
      }
      mo.conf_timeout_s = std::atof(d->conf("mapred.uda.gpu.merge.service.conf.timeout.s", "60").c_str());
      // a task hosted next to an HBM store fetches device descriptors: no pinned fetch arena to prewarm
      // (15 hosted tasks pinning 1 GB each serialized the first wave in the driver, ~150 ms a task)
      if (store_bytes > 0) mo.conf_defaults["mapred.uda.gpu.prewarm.pinned.mb"] = "0";
      Daemon* dp = d.get();
      mo.session_ended = [dp](const std::string& task) {
        std::shared_ptr<DeviceStore> st;
        {
          std::lock_guard<std::mutex> g(dp->mu);
          st = dp->store;
        }
        // whatever a hosted task's descriptors still hold goes with its session
        if (st) st->release_holder("*", gpu::reducer_holder_id(task));
      };
      auto svc = std::make_unique<MergeService>(mo);
      std::lock_guard<std::mutex> g(d->mu);
      d->svc = std::move(svc);
    }
    // what the first wave of hosted tasks would each build on its critical path (code objects, pooled
    // workspaces, shareable pinned delivery rings), built once after READY, long before the first task
    const int warm_tasks = d->svc && !devs.empty()
                               ? (int)std::atoi(d->conf("mapred.uda.daemon.prewarm.tasks", "16").c_str())
                               : 0;
    if (warm_tasks <= 0) d->prewarm_done = 1;  // nothing to build: the node is as warm as it gets
    const int64_t rb = std::atoll(d->conf("mapred.uda.gpu.round.bytes", std::to_string(2ll << 30)).c_str());
    const int64_t kvb = std::atoll(d->conf("mapred.uda.kv.buf.size", std::to_string(1 << 20)).c_str());
    std::string ready;
    put_str(ready, svc_path);
    put<int64_t>(ready, store_bytes);
    d->send(kDReady, ready);
    if (warm_tasks > 0) {
      // the node's first wave spreads over every GPU (and every per-GPU daemon)
      const int per = (warm_tasks + (int)devs.size() * ndaemons - 1) / ((int)devs.size() * ndaemons);
      d->prewarm_tasks = per * (int)devs.size();
      Daemon* dp = d.get();
      d->prewarm = std::thread([dp, devs, per, rb, kvb] {
        name_thread("uda-prewarm");
        const auto t0 = std::chrono::steady_clock::now();
        for (int dv : devs) {
          try {
            prewarm_node_merges(dv, per, rb, 32, kvb);
          } catch (const std::exception& e) {
            UDA_LOG(kWarn, "node daemon: GPU prewarm of device %d: %s", dv, e.what());
          }
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        dp->prewarm_us = (int64_t)(ms * 1e3);
        dp->prewarm_done = 1;
        UDA_LOG(kInfo, "node daemon: prewarmed %d task workspace(s) on %d device(s) in %.0f ms", per, (int)devs.size(), ms);
      });
    }
    std::unique_lock<std::mutex> lk(d->mu);
    d->cv.wait(lk, [&] { return d->closed || d->exit_req; });
  } catch (const std::exception& e) {
    std::string m;
    put_str(m, e.what());
    d->send(kDFailed, m);
    rc = 1;
  }
  // teardown: hosted tasks first (they read the store), then the store
  if (d->prewarm.joinable()) d->prewarm.join();
  {
    std::unique_ptr<MergeService> svc;
    {
      std::lock_guard<std::mutex> g(d->mu);  // the reader adopts connections under it
      svc.swap(d->svc);
    }
    svc.reset();
  }
  {
    std::shared_ptr<DeviceStore> st;
    {
      std::lock_guard<std::mutex> g(d->mu);
      st.swap(d->store);
    }
    st.reset();
  }
  log_set_sink(nullptr, nullptr);
  ::shutdown(ctl_fd, SHUT_RDWR);
  reader.join();
  ::close(ctl_fd);
  return rc;
}

}  // namespace uda

namespace uda {

// ============================================================================ one daemon per GPU

namespace {
// The JSON object (or number) after "key": in `s` ("" if absent). Brace matching: the daemons' stats
// carry no braces inside strings.
std::string json_member(const std::string& s, const std::string& key) {
  const std::string k = "\"" + key + "\":";
  const size_t at = s.find(k);
  if (at == std::string::npos) return "";
  size_t b = at + k.size(), e = b;
  if (b < s.size() && s[b] == '{') {
    int depth = 0;
    for (; e < s.size(); ++e) {
      if (s[e] == '{') ++depth;
      if (s[e] == '}' && --depth == 0) {
        ++e;
        break;
      }
    }
  } else {
    while (e < s.size() && s[e] != ',' && s[e] != '}') ++e;
  }
  return s.substr(b, e - b);
}
int64_t json_int(const std::string& obj, const std::string& key) {
  const std::string v = json_member(obj, key);
  return v.empty() ? 0 : std::atoll(v.c_str());
}

// GPUs of the node as the daemons will number them: the KFD topology's GPU count, or the number of
// entries of HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES when one restricts it. No HIP call: the front
// end lives in the NodeManager and never initialises a GPU runtime.
int visible_gpu_count() {
  int n = (int)usable_gpus().size();
  for (const char* var : {"HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"}) {
    const char* e = std::getenv(var);
    if (!e) continue;
    int k = 0;
    for (const std::string& t : split_list(e)) k += t.empty() ? 0 : 1;
    n = n > 0 ? std::min(n, k) : k;
  }
  return n;
}
}  // namespace

int NodeDaemonSet::node_gpu_count() { return visible_gpu_count(); }

NodeDaemonSet::NodeDaemonSet(const Options& o, Host* host) : opt_(o) {
  const int n = std::max(1, o.count);
  // start them together: each pays a HIP runtime start (seconds on a fresh node)
  std::vector<std::unique_ptr<NodeDaemonClient>> ds((size_t)n);
  std::vector<std::thread> ts;
  for (int i = 0; i < n; ++i)
    ts.emplace_back([&, i] {
      NodeDaemonClient::Options d = o.daemon;
      d.device = n > 1 || o.per_gpu ? i : -1;
      d.ndaemons = n;
      ds[(size_t)i] = std::make_unique<NodeDaemonClient>(d, host);
    });
  for (auto& t : ts) t.join();
  d_ = std::move(ds);
  // the node's merge-service name is the front end's: it routes every client connection to the daemon
  // of the GPU with the fewest live hosted tasks (passing the accepted socket over SCM_RIGHTS)
  if (!opt_.service_path.empty() && (n > 1 || o.per_gpu)) {
    try {
      listen_fd_ = frame::unix_listen(opt_.service_path, 256);
      router_ = std::thread([this] { name_thread("uda-router"); route_main(); });
      UDA_LOG(kInfo, "merge service %s: routing client connections over %d node daemon(s)",
              opt_.service_path.c_str(), n);
    } catch (const std::exception& e) {
      UDA_LOG(kWarn, "merge service %s: cannot listen (%s): reduce tasks merge in their own processes",
              opt_.service_path.c_str(), e.what());
    }
  }
}

NodeDaemonSet::~NodeDaemonSet() {
  stop_ = true;
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (router_.joinable()) router_.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  std::vector<std::thread> ts;
  for (auto& d : d_) ts.emplace_back([&d] { d.reset(); });  // EXIT them together
  for (auto& t : ts) t.join();
}

// Accept, wait (poll) for each connection's first frame header + token, hand it to a daemon. A client
// writes HELLO on its control connection before it opens the data one, so the data connection's token
// is known by the time its DATA_HELLO is read; a connection that says nothing within 10 s is dropped.
void NodeDaemonSet::route_main() {
  struct Pend {
    int fd;
    std::chrono::steady_clock::time_point deadline;
  };
  std::vector<Pend> pend;
  std::map<uint64_t, std::pair<size_t, std::chrono::steady_clock::time_point>> data_route;  // token -> daemon
  while (!stop_) {
    std::vector<pollfd> pf;
    pf.push_back(pollfd{listen_fd_, POLLIN, 0});
    for (auto& p : pend) pf.push_back(pollfd{p.fd, POLLIN, 0});
    (void)::poll(pf.data(), pf.size(), 200);
    if (pf[0].revents & POLLIN) {
      const int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd >= 0) {
        start_trace("router_accept", 0);
        pend.push_back(Pend{fd, std::chrono::steady_clock::now() + std::chrono::seconds(10)});
      }
    }
    const auto now = std::chrono::steady_clock::now();
    for (auto it = data_route.begin(); it != data_route.end();)  // data connections that never came
      it = now > it->second.second ? data_route.erase(it) : std::next(it);
    for (size_t k = 0; k < pend.size();) {
      uint8_t head[16];
      const ssize_t r = ::recv(pend[k].fd, head, sizeof(head), MSG_PEEK | MSG_DONTWAIT);
      bool done = false;
      if (r == (ssize_t)sizeof(head)) {
        uint32_t type;
        uint64_t token;
        std::memcpy(&type, head, 4);
        std::memcpy(&token, head + 8, 8);
        long target = -1;
        if (type == 1) {  // HELLO: the ready daemon with the fewest live sessions
          int best = INT32_MAX;
          for (size_t i = 0; i < d_.size(); ++i)
            if (d_[i] && d_[i]->ready() && d_[i]->live_sessions() < best) {
              best = d_[i]->live_sessions();
              target = (long)i;
            }
          if (target >= 0) data_route[token] = {(size_t)target, now + std::chrono::seconds(30)};
        } else if (type == 6) {  // DATA_HELLO: where its control connection went
          auto it = data_route.find(token);
          if (it != data_route.end()) {
            target = (long)it->second.first;
            data_route.erase(it);
          } else if (now < pend[k].deadline) {
            ++k;  // its HELLO is still being routed
            continue;
          }
        }
        if (target >= 0 && d_[(size_t)target]->adopt(pend[k].fd, type == 1 ? token : 0)) {
          start_trace(type == 1 ? "router_hello" : "router_data", token);
          routed_++;
        } else {
          refused_++;
        }
        done = true;
      } else if (r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) || now > pend[k].deadline) {
        done = true;  // gone, broken or silent
      }
      if (done) {
        ::close(pend[k].fd);  // the daemon holds its own copy now (or nobody wants it)
        pend.erase(pend.begin() + (long)k);
      } else {
        ++k;
      }
    }
  }
  for (auto& p : pend) ::close(p.fd);
}

// A MOF file's store: by a hash of its path, or (that daemon not ready when the file is first asked
// for) the first ready one; remembered, so its releases go where its references are.
size_t NodeDaemonSet::store_of(const std::string& path) {
  if (d_.size() <= 1) return 0;
  std::lock_guard<std::mutex> g(route_mu_);
  auto it = route_.find(path);
  if (it != route_.end()) return it->second;
  size_t i = std::hash<std::string>()(path) % d_.size();
  if (!d_[i]->ready())
    for (size_t k = 0; k < d_.size(); ++k)
      if (d_[(i + k) % d_.size()]->ready()) {
        i = (i + k) % d_.size();
        break;
      }
  route_[path] = i;
  return i;
}

bool NodeDaemonSet::acquire(const std::string& job, const std::string& path, const std::string& holder,
                            int64_t offset, int64_t len, Done done, std::string* why) {
  return d_[store_of(path)]->acquire(job, path, holder, offset, len, std::move(done), why);
}
void NodeDaemonSet::release(const std::string& path, const std::string& holder) {
  d_[store_of(path)]->release(path, holder);
}
void NodeDaemonSet::release_holder(const std::string& job, const std::string& holder) {
  for (auto& d : d_) d->release_holder(job, holder);
}
void NodeDaemonSet::job_over(const std::string& job) {
  for (auto& d : d_) d->job_over(job);
}

std::string NodeDaemonSet::stats_json() {
  std::vector<std::string> js;
  for (auto& d : d_) js.push_back(d->stats_json());
  std::string daemons;
  int64_t sessions = 0, refused = 0, pw_tasks = 0;
  bool pw_done = true, any_pw = false;
  for (size_t i = 0; i < js.size(); ++i) {
    const std::string ms = json_member(js[i], "merge_service"), pw = json_member(js[i], "prewarm");
    sessions += json_int(ms, "sessions");
    refused += json_int(ms, "refused");
    if (!pw.empty()) {
      any_pw = true;
      pw_tasks += json_int(pw, "tasks");
      pw_done = pw_done && json_member(pw, "done") == "true";
    }
    const std::string dm = json_member(js[i], "daemon");
    daemons += (i ? "," : "") + std::string("{\"device\":") + std::to_string(d_[i]->device()) +
               ",\"live_sessions\":" + std::to_string(d_[i]->live_sessions()) +
               (dm.size() > 2 ? "," + dm.substr(1, dm.size() - 2) : std::string()) + "}";
  }
  std::string routing = "\"router\":{\"path\":\"" + opt_.service_path + "\",\"routed\":" + std::to_string(routed_.load()) +
                        ",\"refused\":" + std::to_string(refused_.load()) + ",\"listening\":" +
                        (listen_fd_ >= 0 ? "true" : "false") + "}";
  if (js.size() == 1) {  // one daemon: its own record, plus the per-daemon list and the router
    const std::string& b = js[0];
    return (b.size() > 2 ? b.substr(0, b.size() - 1) + "," : std::string("{")) + "\"daemons\":[" + daemons + "]," +
           routing + "}";
  }
  // several: the node's totals where a caller reads one daemon's fields, and each daemon's full record
  std::string all;
  for (size_t i = 0; i < js.size(); ++i) all += (i ? "," : "") + js[i];
  const std::string d0 = json_member(js[0], "daemon");
  return "{\"daemon\":" + (d0.empty() ? std::string("{}") : d0) + ",\"merge_service\":{\"path\":\"" +
         opt_.service_path + "\",\"sessions\":" + std::to_string(sessions) + ",\"refused\":" + std::to_string(refused) +
         "}" + (any_pw ? ",\"prewarm\":{\"tasks\":" + std::to_string(pw_tasks) + ",\"done\":" + (pw_done ? "true" : "false") + "}" : "") +
         ",\"daemons\":[" + daemons + "]," + routing + ",\"daemon_stats\":[" + all + "]}";
}

}  // namespace uda
