#include "uda/trace.h"

#include <dlfcn.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace uda {
namespace trace {

namespace {
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("UDA_ROCTX");
    if (!e || std::strcmp(e, "1") != 0) return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    r.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    r.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
    if (!r.push || !r.pop) r = Roctx{};
  });
  return r;
}
}  // namespace

void push(const char* name) {
  if (auto f = roctx().push) f(name);
}
void pop() {
  if (auto f = roctx().pop) f();
}
void mark(const char* what) {
  if (auto f = roctx().mark) f(what);
}

namespace {
struct HostEv {
  const char* kind;
  int tid;
  int64_t a, b, t0, t1;
};
struct HostTrace {
  std::mutex mu;
  std::vector<HostEv> ev;
  std::string path;
  std::atomic<bool> on{false};
  HostTrace() {
    if (const char* e = std::getenv("UDA_HOST_TRACE"); e && *e) {
      path = e;
      ev.reserve(1 << 16);
      on = true;
      std::atexit([] { host_dump(); });
    }
  }
};
HostTrace& ht() {
  static HostTrace* t = new HostTrace();  // leaked: used from the atexit hook
  return *t;
}
}  // namespace

bool host_enabled() { return ht().on.load(std::memory_order_relaxed); }

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void host_event(const char* kind, int64_t a, int64_t b, int64_t t0_ns, int64_t t1_ns) {
  HostTrace& t = ht();
  if (!t.on.load(std::memory_order_relaxed)) return;
  const int tid = (int)syscall(SYS_gettid);
  std::lock_guard<std::mutex> g(t.mu);
  t.ev.push_back(HostEv{kind, tid, a, b, t0_ns, t1_ns});
}

void host_dump() {
  HostTrace& t = ht();
  if (!t.on.load()) return;
  std::lock_guard<std::mutex> g(t.mu);
  if (t.ev.empty()) return;
  FILE* f = std::fopen(t.path.c_str(), "a");
  if (!f) return;
  for (const HostEv& e : t.ev)
    std::fprintf(f, "%s,%d,%lld,%lld,%lld,%lld\n", e.kind, e.tid, (long long)e.a, (long long)e.b, (long long)e.t0,
                 (long long)e.t1);
  std::fclose(f);
  t.ev.clear();
}

}  // namespace trace
}  // namespace uda
