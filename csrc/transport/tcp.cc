// TCP transport: multi-process / multi-host fetch path with the reference's message shapes.
//
// Frame = 16-byte netlev header {u8 type, u8 credits, u16 pad, u32 tot_len, u64 src_req}
// (RDMAComm.h:65-72) + payload. Request payload: the RTS string. Response payload:
// u32 ack_len | ACK string | partition bytes (the RDMA WRITE + SEND ack pair of
// RDMAServer.cc:537-631 folded into one frame). Credits: at most `credits` requests in flight per
// connection (wqes_per_conn); the client connects with up to 5 tries (RECONNECT_TRIES).
#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "uda/log.h"
#include "uda/transport.h"
#include "uda/thread_name.h"

namespace uda {

namespace {
constexpr uint8_t kMsgRts = 1;
constexpr uint8_t kMsgAck = 2;
constexpr int kReconnectTries = 5;

struct Header {
  uint8_t type;
  uint8_t credits;
  uint16_t pad;
  uint32_t tot_len;
  uint64_t src_req;
};
static_assert(sizeof(Header) == 16, "netlev header is 16 bytes");

bool read_full(int fd, void* p, size_t n) {
  uint8_t* b = (uint8_t*)p;
  while (n) {
    ssize_t r = ::recv(fd, b, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    b += r;
    n -= (size_t)r;
  }
  return true;
}

bool write_full(int fd, const void* p, size_t n, int flags = 0) {
  const uint8_t* b = (const uint8_t*)p;
  while (n) {
    ssize_t r = ::send(fd, b, n, MSG_NOSIGNAL | flags);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    b += r;
    n -= (size_t)r;
  }
  return true;
}

// Providers of this process by (IPv4 listen address, 0 = any; port). A process that hosts both a
// provider and reduce tasks (the node merge service, set_tcp_local_bypass) serves its tasks' fetches of
// that provider in process: the provider writes straight into the fetch buffer, as on the loopback
// transport, instead of moving every byte through a TCP socket pair.
std::mutex g_local_mu;
std::map<std::pair<uint32_t, int>, DataServer*>& local_servers() {
  static auto* m = new std::map<std::pair<uint32_t, int>, DataServer*>();
  return *m;
}
std::atomic<bool> g_local_bypass{false};

bool local_ipv4(uint32_t ip_be) {
  if ((ntohl(ip_be) >> 24) == 127) return true;
  static const std::vector<uint32_t> mine = [] {
    std::vector<uint32_t> v;
    ifaddrs* ifa = nullptr;
    if (getifaddrs(&ifa) == 0) {
      for (ifaddrs* i = ifa; i; i = i->ifa_next)
        if (i->ifa_addr && i->ifa_addr->sa_family == AF_INET)
          v.push_back(reinterpret_cast<sockaddr_in*>(i->ifa_addr)->sin_addr.s_addr);
      freeifaddrs(ifa);
    }
    return v;
  }();
  return std::find(mine.begin(), mine.end(), ip_be) != mine.end();
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int sz = 4 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof(sz));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof(sz));
}

// ------------------------------------------------------------------------------------ server
class TcpServer : public ServerTransport {
 public:
  TcpServer(int port, int credits, const std::string& bind_addr)
      : port_(port), credits_(credits), bind_addr_(bind_addr) {}
  ~TcpServer() override { stop(); }

  void start(DataServer* s) override {
    server_ = s;
    lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    if (!bind_addr_.empty() && inet_pton(AF_INET, bind_addr_.c_str(), &a.sin_addr) != 1)
      throw std::runtime_error("bad provider bind address '" + bind_addr_ + "'");
    a.sin_port = htons((uint16_t)port_);
    if (::bind(lfd_, (sockaddr*)&a, sizeof(a)) != 0)
      throw std::runtime_error("bind(" + (bind_addr_.empty() ? std::string("*") : bind_addr_) + ":" +
                               std::to_string(port_) + ") failed: " + strerror(errno));
    if (::listen(lfd_, 128) != 0) throw std::runtime_error("listen failed");
    socklen_t len = sizeof(a);
    getsockname(lfd_, (sockaddr*)&a, &len);
    port_ = ntohs(a.sin_port);
    local_key_ = {a.sin_addr.s_addr, port_};
    {
      std::lock_guard<std::mutex> g(g_local_mu);
      local_servers()[local_key_] = s;
    }
    running_ = true;
    acceptor_ = std::thread([this] { name_thread("uda-tcp-accept"); accept_loop(); });
  }

  void stop() override {
    if (!running_.exchange(false)) return;
    {
      std::lock_guard<std::mutex> g(g_local_mu);
      auto it = local_servers().find(local_key_);
      if (it != local_servers().end() && it->second == server_) local_servers().erase(it);
    }
    ::shutdown(lfd_, SHUT_RDWR);
    ::close(lfd_);
    if (acceptor_.joinable()) acceptor_.join();
    std::vector<std::shared_ptr<Conn>> cs;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& c : conns_) ::shutdown(c->fd, SHUT_RDWR);
      cs.swap(conns_);
    }
    // each reader ends once its serves have drained (read_loop), then its socket is closed
    for (auto& c : cs) {
      if (c->reader.joinable()) c->reader.join();
      ::close(c->fd);
    }
  }
  int port() const override { return port_; }

 private:
  // Answers are written by the provider worker that resolved the request (sendfile / send of up to a
  // request's size), so the node's byte serving runs mapred.uda.provider.workers sends at once, in request
  // order. A writer thread per connection was measured too (r6l): 60 connections sending at once shared
  // the box's CPUs fairly, every task's bytes finished late together and the node went from 24.0 to 18.2
  // GB/s (15 tasks, 42.9 GB of declined partitions per wave).
  struct Conn {
    int fd;
    std::mutex mu;  // serializes writes; inflight
    std::condition_variable cv;
    int inflight = 0;
    std::thread reader;
    std::atomic<bool> ended{false};  // the reader returned and no serve is writing to fd
  };
  // Write one answer: header, ack, then the bytes from memory (ptr) or from a file range (sendfile). A
  // failed write shuts the socket down: the client fails the fetches still waiting on it.
  static void answer(const std::shared_ptr<Conn>& c, uint64_t id, const FetchAck& a, const uint8_t* ptr, int fd,
                     int64_t file_off) {
    std::lock_guard<std::mutex> g(c->mu);
    const std::string ack = format_ack(a);
    const uint32_t ack_len = (uint32_t)ack.size();
    const uint64_t data_len = a.status == 0 ? (uint64_t)a.sent : 0;
    Header r{kMsgAck, 1, 0, (uint32_t)(4 + ack_len + data_len), id};
    bool ok = write_full(c->fd, &r, sizeof(r), MSG_MORE) && write_full(c->fd, &ack_len, 4, MSG_MORE) &&
              write_full(c->fd, ack.data(), ack_len, data_len ? MSG_MORE : 0);
    if (ok && data_len) {
      if (ptr) {
        ok = write_full(c->fd, ptr, data_len);
      } else {
        off_t off = (off_t)file_off;
        for (uint64_t left = data_len; ok && left > 0;) {
          const ssize_t w = ::sendfile(c->fd, fd, &off, (size_t)std::min<uint64_t>(left, 1u << 30));
          if (w < 0 && errno == EINTR) continue;
          if (w <= 0) ok = false;  // error, or the file is shorter than its index says
          else left -= (uint64_t)w;
        }
      }
    }
    if (!ok) ::shutdown(c->fd, SHUT_RDWR);
    c->inflight--;
    c->cv.notify_all();
  }

  // Connections whose client went away (one reduce task's, after its fetches): join the reader and
  // close the socket, so a long-lived provider holds threads and descriptors for live clients only.
  void reap_locked() {
    for (auto it = conns_.begin(); it != conns_.end();) {
      if (!(*it)->ended.load()) {
        ++it;
        continue;
      }
      if ((*it)->reader.joinable()) (*it)->reader.join();
      ::close((*it)->fd);
      it = conns_.erase(it);
    }
  }

  void accept_loop() {
    while (running_) {
      int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd < 0) {
        if (!running_) return;
        if (errno == EINTR) continue;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        continue;
      }
      tune(fd);
      auto c = std::make_shared<Conn>();
      c->fd = fd;
      std::lock_guard<std::mutex> g(mu_);
      reap_locked();
      conns_.push_back(c);
      c->reader = std::thread([this, c] {
        read_loop(c);
        std::unique_lock<std::mutex> lk(c->mu);  // serves still answering on this socket finish first
        c->cv.wait(lk, [&] { return c->inflight == 0; });
        c->ended = true;
      });
    }
  }

  void read_loop(const std::shared_ptr<Conn>& c) {
    std::vector<char> payload;
    for (;;) {
      Header h;
      if (!read_full(c->fd, &h, sizeof(h))) return;
      if (h.tot_len > (uint32_t)kFetchReqMax * 4) return;  // protocol violation: drop the connection
      payload.resize(h.tot_len);
      if (h.tot_len && !read_full(c->fd, payload.data(), h.tot_len)) return;
      if (h.type != kMsgRts) continue;
      FetchRequest req;
      if (!parse_rts(std::string(payload.data(), payload.size()), &req, nullptr, nullptr)) continue;
      {
        std::unique_lock<std::mutex> lk(c->mu);
        c->cv.wait(lk, [&] { return c->inflight < credits_; });
        c->inflight++;
      }
      const uint64_t id = h.src_req;
      // by reference first: the provider's memory or the MOF file goes to the socket as it is (send /
      // sendfile), instead of being copied into a chunk and then into the socket
      if (req.buf_len > 0 && server_->serve_ref(req, [c, id](const FetchAck& a, DataServer::Bytes b) {
            answer(c, id, a, b.ptr, b.fd, b.file_off);
            if (b.release) b.release();
          }))
        continue;
      // a chunk of the request's size for the bytes (the provider's registered chunk,
      // NETLEV_RDMA_MEM_CHUNKS_NUM pool); not zero-filled, every byte sent is written first
      std::shared_ptr<uint8_t[]> chunk(new uint8_t[(size_t)std::max<int64_t>(1, req.buf_len)]);
      server_->serve(req, chunk.get(), [c, chunk, id](const FetchAck& a) { answer(c, id, a, chunk.get(), -1, 0); });
    }
  }

  int port_;
  std::string bind_addr_;
  std::pair<uint32_t, int> local_key_{0, 0};
  int credits_;
  int lfd_ = -1;
  std::atomic<bool> running_{false};
  DataServer* server_ = nullptr;
  std::thread acceptor_;
  std::mutex mu_;
  std::vector<std::shared_ptr<Conn>> conns_;
};

// ------------------------------------------------------------------------------------ client
class TcpClient : public ClientTransport {
 public:
  TcpClient(int port, int credits, int connections)
      : port_(port), credits_(credits > 0 ? credits : 1), nconn_(std::max(1, connections)) {}
  ~TcpClient() override { close(); }

  void fetch(const std::string& host, const FetchRequest& req, uint8_t* dst, FetchDone done) override {
    if (g_local_bypass.load()) {
      if (DataServer* s = local_server(host)) {
        if (fault_should_fail_fetch()) {
          FetchAck a;
          a.status = -5;
          a.error = "injected fetch failure";
          done(a);
          return;
        }
        s->serve(req, dst, std::move(done));
        return;
      }
    }
    std::shared_ptr<Conn> c;
    try {
      c = connect(host);
    } catch (const std::exception& e) {
      FetchAck a;
      a.status = -7;
      a.error = e.what();
      done(a);
      return;
    }
    if (fault_should_fail_fetch()) {
      FetchAck a;
      a.status = -5;
      a.error = "injected fetch failure";
      done(a);
      return;
    }
    const uint64_t id = next_id_++;
    std::string rts = format_rts(req, (uint64_t)(uintptr_t)dst, id);
    {
      std::unique_lock<std::mutex> lk(c->mu);
      c->cv.wait(lk, [&] { return c->dead || (int)c->pending.size() < credits_; });
      if (c->dead) {
        lk.unlock();
        FetchAck a;
        a.status = -8;
        a.error = "connection to " + host + " lost";
        done(a);
        return;
      }
      c->pending[id] = Pending{dst, req.buf_len, std::move(done)};
      c->inflight++;
      Header h{kMsgRts, (uint8_t)credits_, 0, (uint32_t)rts.size(), id};
      if (!write_full(c->fd, &h, sizeof(h)) || !write_full(c->fd, rts.data(), rts.size())) {
        c->dead = true;
        ::shutdown(c->fd, SHUT_RDWR);
      }
    }
  }

  void close() override {
    std::vector<std::shared_ptr<Conn>> cs;
    std::vector<std::thread> hs;
    {
      std::lock_guard<std::mutex> g(mu_);
      closing_ = true;
      hs.swap(helpers_);
    }
    for (auto& t : hs) t.join();  // background refills (they install under mu_, into retired_ once closed)
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& kv : hosts_)
        for (auto& c : kv.second.v)
          if (c) cs.push_back(c);
      hosts_.clear();
      for (auto& c : retired_) cs.push_back(c);
      retired_.clear();
      closing_ = false;
    }
    for (auto& c : cs) {
      ::shutdown(c->fd, SHUT_RDWR);
      if (c->reader.joinable()) c->reader.join();
      ::close(c->fd);
    }
  }
  const char* name() const override { return "tcp"; }

 private:
  struct Pending {
    uint8_t* dst;
    int64_t cap;
    FetchDone done;
  };
  struct Conn {
    int fd = -1;
    std::mutex mu;
    std::condition_variable cv;
    std::map<uint64_t, Pending> pending;
    std::atomic<bool> dead{false};
    std::atomic<size_t> inflight{0};  // requests sent, answer not yet read (the least loaded takes the next)
    std::thread reader;
  };

  // The provider of this process that `host_spec` names, if any (resolved once per host).
  DataServer* local_server(const std::string& host_spec) {
    std::pair<uint32_t, int> key{0, -1};
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = resolved_.find(host_spec);
      if (it != resolved_.end()) key = it->second;
    }
    if (key.second < 0) {
      std::string host = host_spec;
      int port = port_;
      const auto colon = host_spec.rfind(':');
      if (colon != std::string::npos) {
        host = host_spec.substr(0, colon);
        port = std::atoi(host_spec.c_str() + colon + 1);
      }
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      uint32_t ip = 0xFFFFFFFFu;  // unresolvable: never local
      if (getaddrinfo(host.c_str(), nullptr, &hints, &res) == 0 && res) {
        ip = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr.s_addr;
        freeaddrinfo(res);
      }
      key = {ip, port};
      std::lock_guard<std::mutex> g(mu_);
      resolved_[host_spec] = key;
    }
    if (key.first == 0xFFFFFFFFu || !local_ipv4(key.first)) return nullptr;
    std::lock_guard<std::mutex> g(g_local_mu);
    auto it = local_servers().find(key);  // a provider listening on exactly that address
    if (it == local_servers().end()) it = local_servers().find({0u, key.second});  // or on any
    return it == local_servers().end() ? nullptr : it->second;
  }

  // The host's connection slots. Connections are opened outside mu_ (an unreachable host costs
  // kReconnectTries tries, ~1.5 s, which must not stall fetches to every other host): one thread at a
  // time opens a host's missing slots while the others use its live connections or wait for the
  // outcome; after a failed open the host is in backoff and fetches to it fail at once.
  struct HostConns {
    std::vector<std::shared_ptr<Conn>> v;
    bool connecting = false;
    std::chrono::steady_clock::time_point backoff_until{};
    std::string last_err;
  };
  static constexpr double kHostBackoffS = 1.0;

  // Open up to `want` connections; stops at the first failure (the host's other slots would fail alike).
  std::vector<std::shared_ptr<Conn>> open_some(const std::string& host_spec, int want, std::string* err) {
    std::vector<std::shared_ptr<Conn>> out;
    for (int k = 0; k < want; ++k) {
      try {
        out.push_back(open_conn(host_spec));
      } catch (const std::exception& e) {
        *err = e.what();
        break;
      }
    }
    return out;
  }

  // Put freshly opened connections into the host's empty slots; record a failure. Under mu_.
  void install(HostConns& hc, std::vector<std::shared_ptr<Conn>>& got, const std::string& err) {
    for (auto& c : hc.v)
      if (!c && !got.empty()) {
        c = std::move(got.back());
        got.pop_back();
      }
    for (auto& c : got) retired_.push_back(c);  // more than the empty slots (close() raced)
    hc.connecting = false;
    if (!err.empty()) {
      hc.last_err = err;
      hc.backoff_until = std::chrono::steady_clock::now() +
                         std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                             std::chrono::duration<double>(kHostBackoffS));
    }
    conn_cv_.notify_all();
  }

  // The live connection to host_spec with the fewest requests in flight.
  std::shared_ptr<Conn> connect(const std::string& host_spec) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      HostConns& hc = hosts_[host_spec];
      if (hc.v.empty()) hc.v.resize((size_t)nconn_);
      std::shared_ptr<Conn> best;
      size_t best_load = SIZE_MAX;
      int missing = 0;
      for (auto& c : hc.v) {
        if (c && c->dead.load()) {
          if (c->reader.joinable()) retired_.push_back(c);  // its reader has failed its requests
          c.reset();
        }
        if (!c) {
          ++missing;
          continue;
        }
        const size_t load = c->inflight.load();
        if (load < best_load) {
          best = c;
          best_load = load;
        }
      }
      const bool may_open = missing > 0 && !hc.connecting && !closing_ &&
                            std::chrono::steady_clock::now() >= hc.backoff_until;
      if (best) {
        if (may_open) {  // refill lost slots in the background; this fetch takes a live connection
          hc.connecting = true;
          helpers_.emplace_back([this, host_spec, missing] {
            std::string err;
            auto got = open_some(host_spec, missing, &err);
            std::lock_guard<std::mutex> g(mu_);
            install(hosts_[host_spec], got, err);
          });
        }
        return best;
      }
      if (may_open) {  // nothing live: this thread opens the host's connections, without mu_
        hc.connecting = true;
        lk.unlock();
        std::string err;
        auto got = open_some(host_spec, missing, &err);
        lk.lock();
        install(hosts_[host_spec], got, err);
        continue;
      }
      if (hc.connecting) {  // another thread is opening them: its outcome is ours
        conn_cv_.wait(lk);
        continue;
      }
      throw std::runtime_error(hc.last_err.empty() ? "cannot connect to " + host_spec : hc.last_err);
    }
  }

  std::shared_ptr<Conn> open_conn(const std::string& host_spec) {
    std::string host = host_spec;
    int port = port_;
    auto colon = host_spec.rfind(':');
    if (colon != std::string::npos) {
      host = host_spec.substr(0, colon);
      port = std::atoi(host_spec.c_str() + colon + 1);
    }
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res)
      throw std::runtime_error("cannot resolve host " + host);
    int fd = -1;
    for (int attempt = 0; attempt < kReconnectTries && fd < 0; ++attempt) {
      fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
        ::close(fd);
        fd = -1;
        std::this_thread::sleep_for(std::chrono::milliseconds(50 << attempt));
      }
    }
    freeaddrinfo(res);
    if (fd < 0) throw std::runtime_error("cannot connect to " + host + ":" + std::to_string(port));
    tune(fd);
    auto c = std::make_shared<Conn>();
    c->fd = fd;
    c->reader = std::thread([c] { name_thread("uda-tcp-read"); reader(c); });
    return c;
  }

  static void reader(std::shared_ptr<Conn> c) {
    std::string ack;
    for (;;) {
      Header h;
      uint32_t ack_len = 0;
      if (!read_full(c->fd, &h, sizeof(h)) || !read_full(c->fd, &ack_len, 4) || ack_len > (1u << 16)) break;
      ack.resize(ack_len);
      if (!read_full(c->fd, &ack[0], ack_len)) break;
      Pending p;
      {
        std::lock_guard<std::mutex> g(c->mu);
        auto it = c->pending.find(h.src_req);
        if (it == c->pending.end()) break;
        p = std::move(it->second);
        c->pending.erase(it);
      }
      c->cv.notify_all();
      // (inflight drops once the bytes are read: a connection still streaming an answer is busy)
      FetchAck a;
      if (!parse_ack(ack, &a)) {
        a.status = -10;
        a.error = "bad ack";
      }
      const uint64_t data_len = (uint64_t)h.tot_len - 4 - ack_len;
      if (data_len > (uint64_t)p.cap || (data_len && !read_full(c->fd, p.dst, data_len))) {
        c->inflight--;
        FetchAck e;
        e.status = -8;
        e.error = "bad or truncated response";
        p.done(e);
        break;
      }
      c->inflight--;
      p.done(a);  // data landed zero-copy in the client buffer
    }
    // connection lost: fail everything pending
    std::map<uint64_t, Pending> left;
    {
      std::lock_guard<std::mutex> g(c->mu);
      c->dead = true;
      left.swap(c->pending);
    }
    c->cv.notify_all();
    for (auto& kv : left) {
      FetchAck a;
      a.status = -8;
      a.error = "connection lost";
      kv.second.done(a);
    }
  }

  int port_;
  int credits_;
  std::atomic<uint64_t> next_id_{1};
  std::mutex mu_;
  int nconn_;
  std::unordered_map<std::string, HostConns> hosts_;
  std::condition_variable conn_cv_;  // a host's open finished
  std::vector<std::thread> helpers_;  // background refills of lost connection slots (joined at close())
  bool closing_ = false;
  std::vector<std::shared_ptr<Conn>> retired_;  // lost connections, joined and closed at close()
  std::unordered_map<std::string, std::pair<uint32_t, int>> resolved_;  // host spec -> (IPv4, port)
};
}  // namespace

void set_tcp_local_bypass(bool on) { g_local_bypass.store(on); }

std::unique_ptr<ServerTransport> make_tcp_server(int port, int credits, const std::string& bind_addr) {
  return std::make_unique<TcpServer>(port, credits > 0 ? credits : 256, bind_addr);
}
std::unique_ptr<ClientTransport> make_tcp_client(int default_port, int credits, int connections) {
  return std::make_unique<TcpClient>(default_port, credits, connections);
}

}  // namespace uda
