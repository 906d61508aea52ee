// Node merge service and its client. See merge_service.h.
#include "merge_service.h"
#include "uda/start_trace.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/un.h>
#include <pwd.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <random>
#include <set>

#include "../consumer/reduce_task.h"
#include "../gpu/sdma.h"
#include "uda/cmd.h"
#include "uda/error.h"
#include "uda/frame.h"
#include "uda/log.h"
#include "uda/transport.h"
#include "uda/thread_name.h"

namespace uda {

namespace {

// ---- framing: u32 type, u32 payload length, payload; an fd may ride along (SCM_RIGHTS). A task uses
// two connections: the control one (HELLO with a session token, commands, configuration, stats, failures)
// and a data one (REGION / DATA from the service, ACK back), so a merged buffer's hand-over costs one
// wake-up on each side instead of a hop through the control reader.
enum Msg : uint32_t {
  kHello = 1,      // c->s: startNative argv, '\0'-separated
  kCmd = 2,        // c->s: command string
  kConfReply = 3,  // c->s: u32 request id, value
  kAck = 4,        // c->s: i32 dataFromUda status
  kExit = 5,       // c->s: reduce task close
  kDataHello = 6,  // c->s, on the task's second (data) connection: u64 session token
  kCmdAsync = 7,   // c->s: a FETCH command; no result frame (a failure is reported as FAIL)
  kReady = 10,     // s->c: task started
  kRefused = 11,     // s->c: HELLO refused (reason)
  kConfReq = 12,   // s->c: u32 request id, key '\0' default
  kRegion = 13,    // s->c: u64 id, u64 bytes, i32 NUMA node + the memfd
  kData = 14,      // s->c: u64 region id, u64 offset, u32 length
  kFetchOver = 15, // s->c
  kFail = 16,      // s->c: reason (failureInUda)
  kCmdResult = 17, // s->c: i32 status, error text
  kStats = 18,     // s->c: stats JSON (reply to EXIT)
};

using frame::get;
using frame::put;
using frame::recv_msg;
using frame::send_msg;
using frame::spin_readable;

}  // namespace

// ============================================================================ service side

struct MergeService::Session : std::enable_shared_from_this<MergeService::Session> {
  MergeService* svc;
  int sock;
  std::mutex send_mu;
  // replies from the client, by kind
  std::mutex mu;
  std::condition_variable cv;
  std::map<uint32_t, std::string> conf_replies;
  uint32_t next_conf = 1;
  bool closed = false;  // the client went away
  // commands run on their own thread: INIT pulls configuration, which the reader thread answers
  std::deque<std::pair<std::string, bool>> cmds;  // (command, async: no result frame)
  bool exit_requested = false;
  std::set<uint64_t> regions_sent;
  uint64_t token = 0;
  std::atomic<int> dsock{-1};  // the data connection (attached by the acceptor, used by the delivering thread)
  // bounce buffer for merged bytes outside shareable pinned memory (EOF tails, host-path buffers)
  int bounce_fd = -1;
  uint8_t* bounce = nullptr;
  size_t bounce_bytes = 0;
  uint64_t bounce_id = 0;
  std::unique_ptr<Host> host;
  std::unique_ptr<ReduceTask> task;
  std::vector<std::string> args;  // startNative arguments (HELLO)
  std::atomic<bool> finished{false};  // the runner has returned: the session can be reaped
  pid_t peer_pid = 0;
  uid_t peer_uid = 0;
  std::thread reader, runner;

  Session(MergeService* s, int fd) : svc(s), sock(fd) {}
  ~Session() {
    if (bounce) munmap(bounce, bounce_bytes);
    if (bounce_fd >= 0) close(bounce_fd);
    if (sock >= 0) close(sock);
    if (dsock.load() >= 0) close(dsock.load());
  }

  bool send(uint32_t type, const std::string& p, int fd = -1) {
    std::lock_guard<std::mutex> g(send_mu);
    return send_msg(sock, type, p, fd);
  }

  // ---- host callbacks of the task (called on the task's threads)
  static int data_cb(void* ctx, const void* buf, int32_t len) { return static_cast<Session*>(ctx)->deliver(buf, len); }
  static int conf_cb(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen) {
    const std::string v = static_cast<Session*>(ctx)->conf(key ? key : "", dflt ? dflt : "");
    const int32_t n = (int32_t)std::min<size_t>(v.size(), (size_t)std::max(0, outlen - 1));
    std::memcpy(out, v.data(), (size_t)n);
    out[n] = 0;
    return n;
  }
  static void fetch_over_cb(void* ctx) { static_cast<Session*>(ctx)->send(kFetchOver, ""); }
  static void failure_cb(void* ctx, const char* reason) {
    static_cast<Session*>(ctx)->send(kFail, reason && *reason ? reason : "merge service task failure");
  }

  std::string conf(const std::string& key, const std::string& dflt_in) {
    const auto od = svc->opt_.conf_defaults.find(key);
    const std::string& dflt = od != svc->opt_.conf_defaults.end() ? od->second : dflt_in;
    uint32_t id;
    {
      std::lock_guard<std::mutex> g(mu);
      if (closed) return dflt;
      id = next_conf++;
    }
    std::string p;
    put<uint32_t>(p, id);
    p += key;
    p.push_back('\0');
    p += dflt;
    if (!send(kConfReq, p)) return dflt;
    std::unique_lock<std::mutex> lk(mu);
    const auto limit = std::chrono::duration<double>(svc->opt_.conf_timeout_s);
    if (!cv.wait_for(lk, limit, [&] { return closed || conf_replies.count(id); })) {
      // a client that stops answering would hold its task (and its HBM reservation) forever: end the
      // session; the task sees the client gone and stops
      UDA_LOG(kError, "merge service: client pid %d did not answer a configuration pull (%s) within %.0f s; "
              "ending its session", (int)peer_pid, key.c_str(), svc->opt_.conf_timeout_s);
      ::shutdown(sock, SHUT_RDWR);
      return dflt;
    }
    if (!conf_replies.count(id)) return dflt;
    std::string v = std::move(conf_replies[id]);
    conf_replies.erase(id);
    return v;
  }

  int deliver(const void* buf, int32_t len) {
    if (dsock < 0 && !data_channel()) return -1;
    gpu::PinnedShare ps;
    uint64_t id;
    size_t off;
    if (len > 0 && gpu::pinned_share_of(buf, (size_t)len, &ps)) {
      if (!regions_sent.count(ps.id)) {  // one delivery thread per task: no race on the set
        std::string r;
        put<uint64_t>(r, ps.id);
        put<uint64_t>(r, ps.region_bytes);
        put<int32_t>(r, ps.numa_node);
        if (!send_msg(dsock, kRegion, r, ps.fd)) return -1;
        regions_sent.insert(ps.id);
      }
      id = ps.id;
      off = ps.offset;
      svc->zero_copy_.fetch_add(1);
    } else {
      if ((size_t)len > bounce_bytes && !grow_bounce((size_t)len)) return -1;
      std::memcpy(bounce, buf, (size_t)len);
      id = bounce_id;
      off = 0;
      svc->bounced_.fetch_add(1);
    }
    std::string d;
    put<uint64_t>(d, id);
    put<uint64_t>(d, off);
    put<uint32_t>(d, (uint32_t)len);
    if (!send_msg(dsock, kData, d)) return -1;
    // the buffer is reused once dataFromUda returns: wait for the client to have consumed it
    uint32_t t;
    std::string a;
    int fd;
    spin_readable(dsock, 200);  // the client copies a 1 MiB buffer in ~30-40 us
    if (!recv_msg(dsock, &t, &a, &fd) || t != kAck) {
      if (fd >= 0) close(fd);
      return -1;
    }
    return get<int32_t>(a, 0);
  }

  bool data_channel() {  // the client attaches it right after HELLO
    std::unique_lock<std::mutex> lk(mu);
    cv.wait_for(lk, std::chrono::seconds(30), [&] { return closed || dsock.load() >= 0; });
    return dsock.load() >= 0;
  }

  bool grow_bounce(size_t need) {
    if (bounce) munmap(bounce, bounce_bytes);
    if (bounce_fd >= 0) close(bounce_fd);
    bounce = nullptr;
    bounce_bytes = 0;
    bounce_fd = (int)memfd_create("uda-bounce", MFD_CLOEXEC);
    const size_t sz = (need + 4095) & ~(size_t)4095;
    if (bounce_fd < 0 || ftruncate(bounce_fd, (off_t)sz) != 0) return false;
    void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, bounce_fd, 0);
    if (p == MAP_FAILED) return false;
    bounce = static_cast<uint8_t*>(p);
    bounce_bytes = sz;
    bounce_id = (1ull << 63) | svc->bounced_.load();  // never a pinned region id; a new id per growth
    std::string r;
    put<uint64_t>(r, bounce_id);
    put<uint64_t>(r, sz);
    put<int32_t>(r, -1);
    return send_msg(dsock, kRegion, r, bounce_fd);
  }

  void start(const std::vector<std::string>& args) {
    uda_callbacks cb{};
    cb.ctx = this;
    cb.data_from_uda = data_cb;
    cb.get_conf = conf_cb;
    cb.fetch_over = fetch_over_cb;
    cb.failure = failure_cb;
    host = std::make_unique<Host>(&cb);
    NetlevOptions opt;
    std::string err;
    if (!parse_options(args, &opt, &err)) throw UdaError("bad startNative options: " + err);
    task = std::make_unique<ReduceTask>(opt, host.get());
    if (svc->opt_.force_device >= 0) task->set_forced_device(svc->opt_.force_device);
    if (peer_uid != ::getuid() && peer_uid != ::geteuid()) {  // a task run for another user: confined
      TaskSandbox sb;
      sb.enabled = true;
      sb.roots = svc->opt_.local_roots;
      task->set_sandbox(sb);
    }
  }

  // The task's whole life on one thread: start (its constructor pulls configuration, which the reader
  // thread answers), the commands in order, and the stop on EXIT or when the client went away.
  void run() {
    try {
      start(args);
    } catch (const std::exception& e) {
      send(kRefused, e.what());
      ::shutdown(sock, SHUT_RDWR);
      finished = true;
      if (svc->opt_.session_closed) svc->opt_.session_closed(token);
      return;
    }
    start_trace("svc_ready", token);
    send(kReady, "");
    svc->sessions_.fetch_add(1);
    run_commands();
    // the task is over, however it ended: whatever its descriptors still hold in this process's HBM
    // store goes (a hosted task's holder id carries this process's pid, which never dies with the task)
    if (svc->opt_.session_ended) {
      const std::string tid = task ? task->task_id() : std::string();
      if (!tid.empty()) {
        try {
          svc->opt_.session_ended(tid);
        } catch (const std::exception& e) {
          UDA_LOG(kWarn, "merge service: session end of %s: %s", tid.c_str(), e.what());
        }
      }
    }
    finished = true;
    if (svc->opt_.session_closed) svc->opt_.session_closed(token);
  }

  void run_commands() {
    for (;;) {
      std::string c;
      bool ex, async = false;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return closed || exit_requested || !cmds.empty(); });
        if (!cmds.empty()) {
          c = std::move(cmds.front().first);
          async = cmds.front().second;
          cmds.pop_front();
          ex = false;
        } else {
          ex = true;
        }
      }
      if (ex) break;
      int32_t st = 0;
      std::string why;
      HadoopCmd hc;
      if (!parse_cmd(c, &hc)) {
        st = -1;
        why = "C++ could not parse Hadoop command";
      } else {
        try {
          task->handle(hc);
        } catch (const std::exception& e) {
          st = -1;
          why = e.what();
        }
      }
      if (async) {  // a FETCH: the client did not wait; its failure is the task's (failureInUda)
        if (st != 0) host->fail(why);
        continue;
      }
      std::string r;
      put<int32_t>(r, st);
      r += why;
      send(kCmdResult, r);
    }
    // EXIT (or the client is gone): stop and join the task, then report its stats
    std::string stats = "{}";
    try {
      task->exit();
      stats = task->stats_json();
    } catch (const std::exception& e) {
      UDA_LOG(kWarn, "merge service: task exit: %s", e.what());
    }
    bool gone;
    {
      std::lock_guard<std::mutex> g(mu);
      gone = closed;
    }
    if (!gone) send(kStats, stats);
  }

  void read_loop() {
    for (;;) {
      uint32_t t;
      std::string p;
      int fd;
      if (!recv_msg(sock, &t, &p, &fd)) break;
      if (fd >= 0) close(fd);
      std::lock_guard<std::mutex> g(mu);
      if (t == kCmd || t == kCmdAsync) {
        cmds.emplace_back(std::move(p), t == kCmdAsync);
      } else if (t == kConfReply) {
        conf_replies[get<uint32_t>(p, 0)] = p.size() > 4 ? p.substr(4) : std::string();
      } else if (t == kExit) {
        exit_requested = true;
      }
      cv.notify_all();
    }
    std::lock_guard<std::mutex> g(mu);
    closed = true;
    if (dsock.load() >= 0) ::shutdown(dsock.load(), SHUT_RDWR);  // a delivery waiting for an ACK returns
    cv.notify_all();
  }
};

MergeService::MergeService(const std::string& path) : MergeService([&] {
        Options o;
        o.path = path;
        return o;
      }()) {}

MergeService::MergeService(const Options& o) : opt_(o) {
  // every shareable pinned allocation keeps its memfd open for the clients that will map it: allow
  // the process as many descriptors as the host lets it have
  rlimit nl{};
  if (getrlimit(RLIMIT_NOFILE, &nl) == 0 && nl.rlim_cur < nl.rlim_max) {
    nl.rlim_cur = nl.rlim_max;
    (void)setrlimit(RLIMIT_NOFILE, &nl);
  }
  gpu::set_pinned_shareable(true);
  set_tcp_local_bypass(true);  // hosted tasks fetch from this process's provider (if any) without a socket
  if (!opt_.path.empty()) listen_fd_ = frame::unix_listen(opt_.path, 256);
  wake_fd_ = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  acceptor_ = std::thread([this] { name_thread("uda-svc-accept"); accept_main(); });
  UDA_LOG(kInfo, "merge service listening on %s (users: %s, max sessions %d)", opt_.path.c_str(), opt_.users.c_str(),
          opt_.max_sessions);
}

MergeService::~MergeService() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
    sess_cv_.notify_all();
  }
  if (listen_fd_ >= 0) ::shutdown(listen_fd_, SHUT_RDWR);
  if (wake_fd_ >= 0) {
    const uint64_t one = 1;
    (void)!::write(wake_fd_, &one, sizeof(one));
  }
  if (acceptor_.joinable()) acceptor_.join();
  {  // adopted after the acceptor's last pass
    std::lock_guard<std::mutex> g(aq_mu_);
    for (int fd : adopted_) ::close(fd);
    adopted_.clear();
  }
  if (wake_fd_ >= 0) ::close(wake_fd_);
  if (listen_fd_ >= 0) close(listen_fd_);
  if (!opt_.path.empty() && opt_.path[0] != '@') ::unlink(opt_.path.c_str());
  std::map<uint64_t, std::thread> shakes;
  std::vector<std::shared_ptr<Session>> live;
  {
    std::lock_guard<std::mutex> g(mu_);
    shakes.swap(shakes_);
  }
  // a handshake still waiting returns within the HELLO timeout (or at once, on stop_, when it waits for
  // its session's registration)
  for (auto& kv : shakes)
    if (kv.second.joinable()) kv.second.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    live.swap(live_);
  }
  for (auto& s : live) {
    ::shutdown(s->sock, SHUT_RDWR);  // the reader sees EOF: the runner stops the task
    if (s->reader.joinable()) s->reader.join();
    if (s->runner.joinable()) s->runner.join();
  }
}

std::string MergeService::default_path(int data_port) { return "@uda-merge-" + std::to_string(data_port); }

bool MergeService::user_allowed(const std::string& users, uid_t uid) {
  if (uid == ::getuid() || uid == ::geteuid()) return true;
  for (size_t b = 0; b <= users.size();) {
    size_t e = users.find(',', b);
    if (e == std::string::npos) e = users.size();
    std::string u = users.substr(b, e - b);
    while (!u.empty() && u.front() == ' ') u.erase(0, 1);
    while (!u.empty() && u.back() == ' ') u.pop_back();
    if (u == "*") return true;
    if (!u.empty()) {
      if (u.find_first_not_of("0123456789") == std::string::npos) {
        if ((uid_t)std::strtoul(u.c_str(), nullptr, 10) == uid) return true;
      } else {
        passwd pw{}, *res = nullptr;
        std::vector<char> buf(16384);
        if (getpwnam_r(u.c_str(), &pw, buf.data(), buf.size(), &res) == 0 && res && res->pw_uid == uid) return true;
      }
    }
    b = e + 1;
  }
  return false;
}

std::string MergeService::stats_json() const {
  return "{\"path\":\"" + opt_.path + "\",\"sessions\":" + std::to_string(sessions_.load()) +
         ",\"refused\":" + std::to_string(refused_.load()) + ",\"zero_copy_buffers\":" +
         std::to_string(zero_copy_.load()) + ",\"bounced_buffers\":" + std::to_string(bounced_.load()) + "}";
}

void MergeService::adopt(int fd) {
  {
    std::lock_guard<std::mutex> g(aq_mu_);
    adopted_.push_back(fd);
  }
  const uint64_t one = 1;
  if (wake_fd_ >= 0) (void)!::write(wake_fd_, &one, sizeof(one));
}

void MergeService::start_handshake(int fd) {
  std::lock_guard<std::mutex> g(mu_);
  if (stop_) {
    ::close(fd);
    return;
  }
  const uint64_t id = next_shake_++;
  shakes_[id] = std::thread([this, fd, id] {
    name_thread("uda-svc-shake");
    handshake(fd);
    std::lock_guard<std::mutex> g2(mu_);
    shakes_done_.insert(id);
  });
}

void MergeService::accept_main() {
  while (!stop_) {
    pollfd pf[2] = {{wake_fd_, POLLIN, 0}, {listen_fd_, POLLIN, 0}};
    // the listener (if any) and adopt()'s wake-ups; the timeout paces the reaping of finished sessions
    const int pr = ::poll(pf, listen_fd_ >= 0 ? 2 : 1, 200);
    if (pr > 0 && (pf[0].revents & POLLIN)) {
      uint64_t n;
      (void)!::read(wake_fd_, &n, sizeof(n));
    }
    std::vector<int> adopted;
    {
      std::lock_guard<std::mutex> g(aq_mu_);
      adopted.swap(adopted_);
    }
    for (int fd : adopted) start_handshake(fd);
    {  // reap finished sessions and handshakes
      // Taken out under mu_, joined and destroyed after it: the last reference to a session runs its
      // reduce task's teardown (pooled workspaces back, pinned rings, streams), ~5-10 ms each, and under
      // mu_ that stalled every adopt() -- and with it the daemon's control channel, descriptor fetches
      // included -- for ~95 ms at the start of each wave of reduce tasks (UDA_START_TRACE, r7a).
      std::vector<std::shared_ptr<Session>> done_sessions;
      std::vector<std::thread> done_shakes;
      {
        std::lock_guard<std::mutex> g(mu_);
        for (auto it = live_.begin(); it != live_.end();) {
          Session& s = **it;
          bool done;
          {
            std::lock_guard<std::mutex> sg(s.mu);
            done = s.closed && s.finished.load();  // joins below return at once
          }
          if (done) {
            done_sessions.push_back(std::move(*it));
            it = live_.erase(it);
          } else {
            ++it;
          }
        }
        for (uint64_t id : shakes_done_) {
          auto t = shakes_.find(id);
          if (t != shakes_.end()) {
            done_shakes.push_back(std::move(t->second));  // it has returned
            shakes_.erase(t);
          }
        }
        shakes_done_.clear();
      }
      for (auto& sp : done_sessions) {
        if (sp->reader.joinable()) sp->reader.join();
        if (sp->runner.joinable()) sp->runner.join();
      }
      done_sessions.clear();
      for (auto& t : done_shakes) t.join();
    }
    if (pr <= 0 || listen_fd_ < 0 || !(pf[1].revents & POLLIN)) continue;
    const int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    // the HELLO is read on a thread of the connection's own: one slow or stalled client never delays
    // another task's admission or its data connection
    start_handshake(fd);
  }
}

void MergeService::handshake(int fd) {
  auto s = std::make_shared<Session>(this, fd);  // ~Session closes the socket unless it is handed on
  // a router (session_closed set) counts the sessions it sent here by their HELLO token: every HELLO
  // that does not become a session reports its end here, a session reports it when its task is over
  struct Closed {
    MergeService* m;
    uint64_t token = 0;
    bool pending = false;
    ~Closed() {
      if (pending && m->opt_.session_closed) m->opt_.session_closed(token);
    }
  } closed_guard{this};
  if (opt_.session_closed) {
    timeval w{(time_t)opt_.hello_timeout_s, 0};
    (void)::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &w, sizeof(w));
    uint8_t head[16];
    if (::recv(fd, head, sizeof(head), MSG_PEEK | MSG_WAITALL) == (ssize_t)sizeof(head)) {
      uint32_t ty;
      std::memcpy(&ty, head, 4);
      if (ty == kHello) {
        std::memcpy(&closed_guard.token, head + 8, 8);
        closed_guard.pending = true;
      }
    }
  }
  uid_t uid = (uid_t)-1;
  pid_t pid = 0;
  if (!frame::peer_cred(fd, &uid, &pid) || !user_allowed(opt_.users, uid)) {
    refused_.fetch_add(1);
    UDA_LOG(kWarn, "merge service: refusing pid %d (uid %d): not in mapred.uda.gpu.merge.service.users (%s)",
            (int)pid, (int)uid, opt_.users.c_str());
    send_msg(fd, kRefused, "uid " + std::to_string((int)uid) + " is not allowed to use the merge service");
    return;
  }
  s->peer_pid = pid;
  s->peer_uid = uid;
  timeval hello_wait{(time_t)opt_.hello_timeout_s, (suseconds_t)((opt_.hello_timeout_s - (time_t)opt_.hello_timeout_s) * 1e6)};
  (void)::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &hello_wait, sizeof(hello_wait));
  uint32_t t;
  std::string p;
  int pfd;
  if (!recv_msg(fd, &t, &p, &pfd) || (t != kHello && t != kDataHello) || p.size() < 8) {
    if (pfd >= 0) close(pfd);
    return;
  }
  timeval none{0, 0};
  (void)::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &none, sizeof(none));
  const uint64_t token = get<uint64_t>(p, 0);
  start_trace(t == kDataHello ? "svc_data_hello" : "svc_hello", token);
  if (t == kDataHello) {  // a task's data connection: attach it to its session (same peer process)
    // the control connection's handshake (its own thread) may not have registered the session yet
    std::shared_ptr<Session> owner;
    {
      std::unique_lock<std::mutex> g(mu_);
      sess_cv_.wait_for(g, std::chrono::duration<double>(opt_.hello_timeout_s), [&] {
        for (auto& x : live_)
          if (x->token == token && x->peer_pid == pid) owner = x;
        return owner != nullptr || stop_.load();
      });
    }
    if (owner) {
      std::lock_guard<std::mutex> g(owner->mu);
      if (owner->dsock.load() < 0 && !owner->closed) {
        owner->dsock.store(s->sock);
        s->sock = -1;  // now the owner's
        owner->cv.notify_all();
      }
    }
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    int running = 0, mine = 0;
    for (auto& x : live_) {
      if (x->finished.load()) continue;
      ++running;
      mine += x->peer_uid == uid ? 1 : 0;
    }
    const bool foreign = uid != ::getuid() && uid != ::geteuid();
    if (stop_ || running >= opt_.max_sessions || (foreign && mine >= opt_.max_sessions_per_user)) {
      refused_.fetch_add(1);
      send_msg(fd, kRefused, stop_ ? std::string("merge service stopping")
                             : running >= opt_.max_sessions
                                 ? "merge service full (" + std::to_string(running) + " hosted tasks)"
                                 : "uid " + std::to_string((int)uid) + " already has " + std::to_string(mine) +
                                       " hosted tasks");
      return;
    }
    s->token = token;
    p.erase(0, 8);
    for (size_t b = 0; b < p.size();) {
      const size_t e = p.find('\0', b);
      s->args.push_back(p.substr(b, e == std::string::npos ? std::string::npos : e - b));
      if (e == std::string::npos) break;
      b = e + 1;
    }
    s->reader = std::thread([s] { name_thread("uda-svc-read"); s->read_loop(); });
    s->runner = std::thread([s] { name_thread("uda-svc-run"); s->run(); });
    closed_guard.pending = false;  // the session reports its own end
    live_.push_back(s);
    sess_cv_.notify_all();
  }
}

// ============================================================================ client side

struct RemoteReduceTask::Impl {
  Host* host;
  int sock = -1, dsock = -1;
  int bound_node = -1;  // NUMA node the data thread is bound to (the delivery rings' node)
  std::thread reader, data_reader;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<int32_t, std::string>> results;
  bool have_stats = false, closed = false, exited = false, refused = false;
  std::string stats = "{}";
  std::map<uint64_t, std::pair<uint8_t*, size_t>> regions;  // id -> our mapping

  ~Impl() {
    if (sock >= 0) ::shutdown(sock, SHUT_RDWR);
    if (dsock >= 0) ::shutdown(dsock, SHUT_RDWR);
    if (reader.joinable()) reader.join();
    if (data_reader.joinable()) data_reader.join();
    if (sock >= 0) close(sock);
    if (dsock >= 0) close(dsock);
    for (auto& kv : regions) munmap(kv.second.first, kv.second.second);
  }

  // The data connection: REGION (a shared mapping to add) and DATA (a merged buffer in one of them)
  // from the service, in order; each DATA is handed to dataFromUda in place, then acknowledged. Waits
  // briefly with a spin first: the next buffer usually follows the ACK within microseconds.
  void data_loop() {
    for (;;) {
      spin_readable(dsock, 100);
      uint32_t t;
      std::string p;
      int fd;
      if (!recv_msg(dsock, &t, &p, &fd)) return;
      if (t == kRegion) {
        const uint64_t id = get<uint64_t>(p, 0), bytes = get<uint64_t>(p, 8);
        const int node = p.size() >= 20 ? get<int32_t>(p, 16) : -1;
        if (node >= 0 && node != bound_node) {
          // dataFromUda copies out of these pages: run where they live, as the in-process delivery
          // thread does (gpu_merge.cc binds it to the GPU's node)
          gpu::bind_thread_to_numa(node);
          bound_node = node;
        }
        if (fd >= 0) {
          // populated up front: faulting the pages in one at a time as the buffers arrive costs a
          // minor fault per 4 KiB (shared memory pages are small unless the host enables THP for shmem)
          void* m = mmap(nullptr, bytes, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
          if (m != MAP_FAILED) (void)madvise(m, bytes, MADV_HUGEPAGE);
          close(fd);
          if (m != MAP_FAILED) {
            auto old = regions.find(id);
            if (old != regions.end()) munmap(old->second.first, old->second.second);
            regions[id] = {static_cast<uint8_t*>(m), (size_t)bytes};
          }
        }
      } else if (t == kData) {
        if (fd >= 0) close(fd);
        const uint64_t id = get<uint64_t>(p, 0), off = get<uint64_t>(p, 8);
        const uint32_t len = get<uint32_t>(p, 16);
        int32_t st = -1;
        auto it = regions.find(id);
        if (it != regions.end() && off + len <= it->second.second)
          st = host->data_from_uda(it->second.first + off, (int32_t)len);
        else
          host->fail("merge service sent a buffer outside its shared regions");
        std::string a;
        put<int32_t>(a, st);
        if (!send_msg(dsock, kAck, a)) return;
      } else if (fd >= 0) {
        close(fd);
      }
    }
  }

  void read_loop() {
    for (;;) {
      uint32_t t;
      std::string p;
      int fd;
      if (!recv_msg(sock, &t, &p, &fd)) break;
      if (t == kConfReq) {
        if (fd >= 0) close(fd);
        const uint32_t id = get<uint32_t>(p, 0);
        const std::string kd = p.size() > 4 ? p.substr(4) : std::string();
        const size_t z = kd.find('\0');
        const std::string key = kd.substr(0, z), dflt = z == std::string::npos ? "" : kd.substr(z + 1);
        std::string r;
        put<uint32_t>(r, id);
        r += host->get_conf(key, dflt);
        std::lock_guard<std::mutex> g(send_mu);
        if (!send_msg(sock, kConfReply, r)) break;
      } else {
        if (fd >= 0) close(fd);
        if (t == kFetchOver) {
          host->fetch_over();
        } else if (t == kFail) {
          host->fail(p);
        } else {
          std::lock_guard<std::mutex> g(mu);
          if (t == kCmdResult) {
            results.emplace_back(get<int32_t>(p, 0), p.size() > 4 ? p.substr(4) : std::string());
          } else if (t == kStats) {
            stats = p;
            have_stats = true;
          } else if (t == kReady) {
            results.emplace_back(0, std::string());
          } else if (t == kRefused) {
            results.emplace_back(-1, p);
            refused = true;  // the start fails in the constructor: no task to report a failure for
          }
          cv.notify_all();
        }
      }
    }
    std::lock_guard<std::mutex> g(mu);
    const bool unexpected = !exited && !refused;
    closed = true;
    cv.notify_all();
    if (unexpected) host->fail("merge service connection lost");
  }

  std::pair<int32_t, std::string> wait_result() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return closed || !results.empty(); });
    if (results.empty()) return {-1, "merge service connection lost"};
    auto r = std::move(results.front());
    results.pop_front();
    return r;
  }

  bool send(uint32_t t, const std::string& p) {
    std::lock_guard<std::mutex> g(send_mu);
    return send_msg(sock, t, p);
  }
  std::mutex send_mu;
};

// The service end of a connection must run as our own user, root, or a user the job names
// (mapred.uda.gpu.merge.service.server.users): an abstract socket name is open to anyone to bind first.
static void check_service_peer(int fd, const std::string& path, const std::string& server_users) {
  uid_t uid = (uid_t)-1;
  pid_t pid = 0;
  if (!frame::peer_cred(fd, &uid, &pid)) throw UdaError("merge service " + path + ": no peer credentials");
  if (uid == 0 || MergeService::user_allowed(server_users, uid)) return;
  throw UdaError("merge service " + path + " is served by uid " + std::to_string((int)uid) + " (pid " +
                 std::to_string((int)pid) + "), not a trusted user (mapred.uda.gpu.merge.service.server.users)");
}

RemoteReduceTask::RemoteReduceTask(const std::string& path, const std::vector<std::string>& args, Host* host)
    : impl_(new Impl) {
  impl_->host = host;
  start_trace("client_begin", 0);
  const std::string server_users = host->get_conf("mapred.uda.gpu.merge.service.server.users", "");
  impl_->sock = frame::unix_connect(path);
  if (impl_->sock < 0) throw UdaError("merge service " + path + " not reachable: " + strerror(errno));
  check_service_peer(impl_->sock, path, server_users);
  uint64_t token = 0;
  {
    std::random_device rd;
    token = ((uint64_t)rd() << 32) ^ rd() ^ ((uint64_t)getpid() << 20);
  }
  std::string hello;
  put<uint64_t>(hello, token);
  for (size_t i = 0; i < args.size(); ++i) {
    if (i) hello.push_back('\0');
    hello += args[i];
  }
  if (!send_msg(impl_->sock, kHello, hello)) throw UdaError("merge service " + path + ": HELLO failed");
  start_trace("client_hello_sent", token);
  impl_->dsock = frame::unix_connect(path);
  if (impl_->dsock >= 0) check_service_peer(impl_->dsock, path, server_users);
  std::string dh;
  put<uint64_t>(dh, token);
  if (impl_->dsock < 0 || !send_msg(impl_->dsock, kDataHello, dh))
    throw UdaError("merge service " + path + ": data connection failed");
  Impl* im = impl_.get();
  impl_->data_reader = std::thread([im] { im->data_loop(); });
  impl_->reader = std::thread([im] { im->read_loop(); });
  start_trace("client_data_sent", token);
  const auto r = impl_->wait_result();
  start_trace("client_ready", token);
  if (r.first != 0) {
    {
      std::lock_guard<std::mutex> g(impl_->mu);
      impl_->exited = true;  // a refused start is an error of this call, not a task failure
    }
    throw UdaError("merge service refused the task: " + r.second);
  }
}

RemoteReduceTask::~RemoteReduceTask() {
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    impl_->exited = true;
  }
  impl_.reset();
}

void RemoteReduceTask::handle(const std::string& cmd) {
  // FETCH commands do not wait for the service (a task's 32+ FETCHes arrive back to back and each
  // round trip costs two thread wake-ups on a loaded node); the reference queues them on the native
  // side too. INIT / FINAL / EXIT stay synchronous: their errors belong to the call.
  HadoopCmd c;
  if (parse_cmd(cmd, &c) && c.header == kFetchMsg) {
    if (!impl_->send(kCmdAsync, cmd)) throw UdaError("merge service connection lost");
    return;
  }
  if (!impl_->send(kCmd, cmd)) throw UdaError("merge service connection lost");
  const auto r = impl_->wait_result();
  if (r.first != 0) throw UdaError(r.second);
}

void RemoteReduceTask::exit() {
  {
    std::lock_guard<std::mutex> g(impl_->mu);
    if (impl_->exited) return;
    impl_->exited = true;
  }
  if (impl_->send(kExit, "")) {
    std::unique_lock<std::mutex> lk(impl_->mu);
    impl_->cv.wait_for(lk, std::chrono::seconds(120), [&] { return impl_->have_stats || impl_->closed; });
  }
  // the session is over: nothing more comes on either connection, so the readers go now (the JVM
  // keeps a closed reduce task's handle until it is collected)
  ::shutdown(impl_->sock, SHUT_RDWR);
  ::shutdown(impl_->dsock, SHUT_RDWR);
  if (impl_->reader.joinable()) impl_->reader.join();
  if (impl_->data_reader.joinable()) impl_->data_reader.join();
}

std::string RemoteReduceTask::stats_json() {
  std::lock_guard<std::mutex> g(impl_->mu);
  if (impl_->have_stats && impl_->stats.size() > 1 && impl_->stats.back() == '}')
    return impl_->stats.substr(0, impl_->stats.size() - 1) + ",\"merge_service\":true}";
  return impl_->stats;
}

}  // namespace uda
