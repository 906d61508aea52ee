#include "uda/fault.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

namespace uda {

namespace {
struct ThreadFaults {
  std::map<std::string, std::pair<long, long>> sites;  // site -> (n, hits)
};
thread_local ThreadFaults* t_faults = nullptr;
}  // namespace

FaultScope::FaultScope(const std::string& spec) : prev_(t_faults) {
  if (spec.empty()) return;
  auto* f = new ThreadFaults;
  for (size_t b = 0; b <= spec.size();) {
    size_t e = spec.find(',', b);
    if (e == std::string::npos) e = spec.size();
    const std::string kv = spec.substr(b, e - b);
    const size_t eq = kv.find('=');
    if (eq != std::string::npos && eq > 0) f->sites[kv.substr(0, eq)] = {std::atol(kv.c_str() + eq + 1), 0};
    b = e + 1;
  }
  t_faults = f;
}

FaultScope::~FaultScope() {
  if (t_faults != prev_) delete t_faults;
  t_faults = static_cast<ThreadFaults*>(prev_);
}

bool fault_hit(const char* site) {
  if (ThreadFaults* f = t_faults) {  // this thread's own spec replaces the environment's for its sites
    auto it = f->sites.find(site);
    if (it != f->sites.end()) return it->second.first > 0 && ++it->second.second == it->second.first;
  }
  const std::string var = std::string("UDA_FAULT_") + site;
  const char* e = std::getenv(var.c_str());
  static std::mutex mu;
  static std::map<std::string, std::pair<std::string, long>> state;  // site -> (spec, count)
  std::lock_guard<std::mutex> g(mu);
  if (!e || !*e) {  // unset: the next arming counts from zero again
    state.erase(var);
    return false;
  }
  auto& st = state[var];
  if (st.first != e) st = {e, 0};
  const long n = std::atol(e);
  return n > 0 && ++st.second == n;
}

}  // namespace uda
