// In-process loopback transport: the provider writes straight into the consumer's buffer (the
// one-sided RDMA WRITE analogue) and completes the request through the same callback path.
#include <mutex>
#include <unordered_map>

#include "uda/log.h"
#include "uda/transport.h"

namespace uda {

namespace {
std::mutex g_mu;
std::unordered_map<std::string, DataServer*>& registry() {
  static std::unordered_map<std::string, DataServer*> r;
  return r;
}

class LoopbackClient : public ClientTransport {
 public:
  void fetch(const std::string& host, const FetchRequest& req, uint8_t* dst, FetchDone done) override {
    DataServer* s = nullptr;
    {
      std::lock_guard<std::mutex> g(g_mu);
      auto it = registry().find(host);
      if (it == registry().end()) it = registry().find("*");  // single-provider wildcard
      if (it != registry().end()) s = it->second;
    }
    if (!s) {
      FetchAck a;
      a.status = -2;
      a.error = "no loopback provider for host " + host;
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
    s->serve(req, dst, std::move(done));
  }
  const char* name() const override { return "loopback"; }
};

class LoopbackServer : public ServerTransport {
 public:
  explicit LoopbackServer(std::string host) : host_(std::move(host)) {}
  ~LoopbackServer() override { stop(); }
  void start(DataServer* s) override {
    server_ = s;
    loopback_register(host_, s);
  }
  void stop() override {
    if (server_) loopback_unregister(host_, server_);
    server_ = nullptr;
  }

 private:
  std::string host_;
  DataServer* server_ = nullptr;
};
}  // namespace

void loopback_register(const std::string& host, DataServer* server) {
  std::lock_guard<std::mutex> g(g_mu);
  registry()[host] = server;
}

void loopback_unregister(const std::string& host, DataServer* server) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = registry().find(host);
  if (it != registry().end() && it->second == server) registry().erase(it);
}

std::unique_ptr<ClientTransport> make_loopback_client() { return std::make_unique<LoopbackClient>(); }
std::unique_ptr<ServerTransport> make_loopback_server(const std::string& host) {
  return std::make_unique<LoopbackServer>(host);
}

}  // namespace uda
