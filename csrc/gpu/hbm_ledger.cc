// Per-device HBM byte budget. See hbm_ledger.h.
#include "hbm_ledger.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>

#include "uda/error.h"
#include "uda/log.h"
#include "uda/node_registry.h"

namespace uda {
namespace gpu {

namespace {
thread_local HbmLedger::Reservation* tls_res = nullptr;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

std::string mb(int64_t b) {
  char s[32];
  std::snprintf(s, sizeof(s), "%.2f GB", (double)b / 1e9);
  return s;
}
}  // namespace

std::string device_key(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess && bus[0]) return bus;
  (void)hipGetLastError();
  return "hip-device-" + std::to_string(device);
}

std::vector<std::string> visible_device_keys() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  std::vector<std::string> keys;
  for (int i = 0; i < n; ++i) keys.push_back(device_key(i));
  return keys;
}

HbmLedger& HbmLedger::get() {
  static HbmLedger* l = new HbmLedger;  // never destroyed: buffers may be freed during static teardown
  return *l;
}

HbmLedger::Dev& HbmLedger::dev(int device) {
  Dev& d = devs_[device];
  if (d.init) return d;
  d.init = true;
  d.key = device_key(device);
  size_t total = 0;
  if (hipDeviceTotalMem(&total, device) != hipSuccess) {
    (void)hipGetLastError();
    total = 0;
  }
  d.total = (int64_t)total;
  d.budget = d.total > 0 ? (int64_t)((double)d.total * kDefaultFraction) : INT64_MAX / 4;
  return d;
}

void HbmLedger::set_fake_device(int device, int64_t total_bytes, const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = devs_[device];
  d.init = true;
  d.fake = true;
  d.key = key;
  d.total = total_bytes;
  d.budget = (int64_t)((double)total_bytes * kDefaultFraction);
}

void HbmLedger::set_fake_untracked(int device, int64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  devs_[device].fake_untracked = bytes;
}

void HbmLedger::configure(int device, double conf) {
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = dev(device);
  if (conf > 1.0) {
    d.budget = (int64_t)conf;
  } else {
    const double f = conf > 0 ? conf : kDefaultFraction;
    d.budget = d.total > 0 ? (int64_t)((double)d.total * f) : INT64_MAX / 4;
  }
  cv_.notify_all();
}

int64_t HbmLedger::budget(int device) {
  std::lock_guard<std::mutex> g(mu_);
  return dev(device).budget;
}

void HbmLedger::publish(Dev& d) {
  if (NodeRegistry* r = NodeRegistry::instance()) {
    try {
      r->set_bytes(d.key, d.used + d.reserved, d.resident);
    } catch (const std::exception&) {
    }
  }
}

int64_t HbmLedger::others(Dev& d) {
  NodeRegistry* r = NodeRegistry::instance();
  if (!r) return 0;
  try {
    const NodeRegistry::Use u = r->usage(d.key);
    return std::max<int64_t>(0, u.bytes - (d.used + d.reserved));
  } catch (const std::exception&) {
    return 0;
  }
}

int64_t HbmLedger::others_resident(Dev& d) {
  NodeRegistry* r = NodeRegistry::instance();
  if (!r) return 0;
  try {
    const NodeRegistry::Use u = r->usage(d.key);
    return std::max<int64_t>(0, u.resident - d.resident);
  } catch (const std::exception&) {
    return 0;
  }
}

int64_t HbmLedger::device_used(int device, Dev& d) {
  if (d.fake) return d.fake_untracked > 0 ? d.fake_untracked + others(d) + d.used : 0;
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  size_t free_b = 0, total_b = 0;
  const bool ok = (cur == device || hipSetDevice(device) == hipSuccess) && hipMemGetInfo(&free_b, &total_b) == hipSuccess;
  if (cur != device) (void)hipSetDevice(cur);
  if (!ok) {
    (void)hipGetLastError();
    return 0;
  }
  const int64_t u = (int64_t)(total_b - free_b);
  d.device_peak = std::max(d.device_peak, u);
  return u;
}

void HbmLedger::add_pool(Pool p) {
  std::lock_guard<std::mutex> g(pools_mu_);
  pools_.push_back(std::move(p));
}

int64_t HbmLedger::trim_pools(int device, int64_t want) {
  std::vector<Pool> ps;
  {
    std::lock_guard<std::mutex> g(pools_mu_);
    ps = pools_;
  }
  int64_t freed = 0;
  // largest idle pool first: each pool frees its own largest idle objects first
  std::sort(ps.begin(), ps.end(), [device](const Pool& a, const Pool& b) { return a.idle(device) > b.idle(device); });
  for (auto& p : ps) {
    if (freed >= want) break;
    freed += p.trim(device, want - freed);
  }
  if (freed > 0) {
    std::lock_guard<std::mutex> g(mu_);
    dev(device).trimmed += freed;
  }
  return freed;
}

int64_t HbmLedger::idle_bytes(int device) {
  std::vector<Pool> ps;
  {
    std::lock_guard<std::mutex> g(pools_mu_);
    ps = pools_;
  }
  int64_t n = 0;
  for (auto& p : ps) n += p.idle(device);
  return n;
}

void HbmLedger::on_alloc(int device, int64_t bytes, bool resident) {
  if (bytes <= 0) return;
  std::unique_lock<std::mutex> lk(mu_);
  Dev& d = dev(device);
  Reservation* r = tls_res;
  if (!resident && r && r->device_ == device && r->left_ > 0) {
    const int64_t take = std::min(r->left_, bytes);
    r->left_ -= take;
    d.reserved -= take;
    bytes -= take;
    d.used += take;
  }
  if (bytes > 0) {
    int64_t over = others(d) + d.used + d.reserved + bytes - d.budget;
    if (over > 0) {
      lk.unlock();
      trim_pools(device, over);
      lk.lock();
      over = others(d) + d.used + d.reserved + bytes - d.budget;
    }
    if (over > 0) {
      d.over += bytes;
      UDA_LOG(kWarn, "HBM budget of device %d exceeded by %s (allocation of %s outside a reservation)", device,
              mb(over).c_str(), mb(bytes).c_str());
    }
    d.used += bytes;
    if (resident) d.resident += bytes;
  }
  d.peak = std::max(d.peak, d.used + d.reserved);
  publish(d);
}

void HbmLedger::on_free(int device, int64_t bytes, bool resident) {
  if (bytes <= 0) return;
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = dev(device);
  d.used -= bytes;
  if (resident) d.resident -= bytes;
  publish(d);
  cv_.notify_all();
}

HbmLedger::Reservation* HbmLedger::bound() { return tls_res; }

int64_t HbmLedger::used(int device) {
  std::lock_guard<std::mutex> g(mu_);
  return dev(device).used;
}

int64_t HbmLedger::headroom(int device) {
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = dev(device);
  // what stays whatever the tasks do: MOF stores of every process on the node, and the device memory no
  // ledger knows about (HIP runtime, code objects, allocations outside libuda). The latter is what the
  // device reports in use beyond every process's tracked bytes; reserve() admits against the device's
  // own figure too, so a round sized from a headroom without it could pass here and never be granted.
  return d.budget - others_resident(d) - d.resident - untracked(device, d);
}

int64_t HbmLedger::untracked(int device, Dev& d) {
  const int64_t dev_used = device_used(device, d);
  if (dev_used <= 0) return 0;
  // others() counts the other processes' reservations too (not yet allocated): this underestimates the
  // untracked bytes a little, which only lets a task try a round the admission check may still refuse
  return std::max<int64_t>(0, dev_used - (others(d) + d.used));
}

std::unique_ptr<HbmLedger::Reservation> HbmLedger::reserve(int device, int64_t bytes, const std::function<bool()>& stop,
                                                           double timeout_s) {
  std::unique_ptr<Reservation> res(new Reservation);
  res->device_ = device;
  res->prev_bound_ = tls_res;
  tls_res = res.get();
  if (bytes <= 0) return res;
  const double t0 = now_ms();
  const int64_t hr = headroom(device);
  if (bytes > hr)
    throw HbmBudgetError("device working set of " + mb(bytes) + " exceeds the HBM budget headroom of device " +
                         std::to_string(device) + " (" + mb(hr) + ")");
  std::unique_lock<std::mutex> lk(mu_);
  Dev& d = dev(device);
  const uint64_t me = d.next_ticket++;
  d.queue.push_back(me);
  bool waited = false;
  auto leave = [&] {
    d.queue.erase(std::find(d.queue.begin(), d.queue.end(), me));
    cv_.notify_all();
  };
  for (;;) {
    if (d.queue.front() == me) {
      // the ledger's own accounting, and what the device itself reports in use (the HIP runtime's and
      // any untracked allocations count against the budget too) plus the reservations not yet allocated
      const int64_t over = std::max(others(d) + d.used + d.reserved + bytes - d.budget,
                                    device_used(device, d) + d.reserved + bytes - d.budget);
      if (over <= 0) break;
      lk.unlock();
      const int64_t freed = trim_pools(device, over);
      lk.lock();
      if (freed > 0) continue;
      // nothing that could ever be freed is held: no reservation of this process, no working set of a
      // running task here or in another process, no idle pooled object left. Waiting would only hold
      // every later reservation of the device behind this one for the whole timeout.
      if (d.reserved == 0 && d.used - d.resident <= 0 && others(d) - others_resident(d) <= 0) {
        leave();
        throw HbmBudgetError("a " + mb(bytes) + " working set never fits on device " + std::to_string(device) +
                             ": " + mb(device_used(device, d)) + " in use by the device's resident data and " +
                             "untracked allocations, budget " + mb(d.budget));
      }
    }
    if (stop && stop()) {
      leave();
      throw HbmBudgetError("reduce task stopped while waiting for HBM");
    }
    if (now_ms() - t0 > timeout_s * 1000.0) {
      leave();
      throw HbmBudgetError("no HBM for a " + mb(bytes) + " working set on device " + std::to_string(device) +
                           " within " + std::to_string((int)timeout_s) + " s");
    }
    waited = true;
    // other processes free memory without notifying us: poll
    cv_.wait_for(lk, std::chrono::milliseconds(5));
  }
  d.queue.pop_front();
  d.reserved += bytes;
  d.peak = std::max(d.peak, d.used + d.reserved);
  res->granted_ = res->left_ = bytes;
  res->wait_ms_ = now_ms() - t0;
  if (waited) {
    ++d.waits;
    d.wait_ms += res->wait_ms_;
  }
  publish(d);
  cv_.notify_all();
  return res;
}

HbmLedger::Reservation::~Reservation() {
  unbind();
  if (left_ > 0) {
    HbmLedger& l = HbmLedger::get();
    std::lock_guard<std::mutex> g(l.mu_);
    Dev& d = l.dev(device_);
    d.reserved -= left_;
    left_ = 0;
    l.publish(d);
    l.cv_.notify_all();
  }
}

HbmLedger::Reservation::Scope HbmLedger::Reservation::bind() {
  Reservation* prev = tls_res;
  tls_res = this;
  return Scope(prev);
}

HbmLedger::Reservation::Scope::~Scope() { tls_res = prev; }

void HbmLedger::Reservation::unbind() {
  if (tls_res == this) tls_res = prev_bound_;
  prev_bound_ = nullptr;
}

void HbmLedger::reset_peak(int device) {
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = dev(device);
  d.peak = d.used + d.reserved;
}

HbmLedger::Stats HbmLedger::stats(int device) {
  std::lock_guard<std::mutex> g(mu_);
  Dev& d = dev(device);
  Stats s;
  s.budget = d.budget;
  s.used = d.used;
  s.reserved = d.reserved;
  s.peak = d.peak;
  s.resident = d.resident;
  s.node_bytes = others(d) + d.used + d.reserved;
  s.trimmed = d.trimmed;
  s.over = d.over;
  s.device_peak = d.device_peak;
  s.waits = d.waits;
  s.wait_ms = d.wait_ms;
  return s;
}

}  // namespace gpu
}  // namespace uda
