#include "uda/trace.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

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

}  // namespace trace
}  // namespace uda
