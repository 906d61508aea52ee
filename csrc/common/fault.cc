#include "uda/fault.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <string>

namespace uda {

bool fault_hit(const char* site) {
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
