// Error type and failure funnel.
//
// Parity: `UdaException` (src/include/IOUtility.h:174-180) and the fallback contract: any native
// failure reaches the host once through `failureInUda` (src/UdaBridge.cc:506-530) so the host can
// fall back to its vanilla shuffle. Here every engine thread funnels exceptions into
// `report_failure()`, which invokes the registered failure hook exactly once per owner.
#pragma once
#include <atomic>
#include <functional>
#include <stdexcept>
#include <string>

namespace uda {

class UdaError : public std::runtime_error {
 public:
  explicit UdaError(const std::string& what) : std::runtime_error(what) {}
};

// Raised on caller-visible protocol/config errors (bad command, unsupported key class ...).
class ProtocolError : public UdaError {
 public:
  using UdaError::UdaError;
};

// A device working set that does not fit the HBM budget (mapred.uda.gpu.hbm.budget) now, or ever.
class HbmBudgetError : public UdaError {
 public:
  using UdaError::UdaError;
};

// A one-shot failure latch: the first report wins and triggers the hook; later ones are counted.
class FailureLatch {
 public:
  void set_hook(std::function<void(const std::string&)> hook) { hook_ = std::move(hook); }
  // Returns true if this call was the first failure.
  bool report(const std::string& why);
  bool failed() const { return failed_.load(); }
  int count() const { return count_.load(); }
  const std::string& first_reason() const { return reason_; }

 private:
  std::function<void(const std::string&)> hook_;
  std::atomic<bool> failed_{false};
  std::atomic<int> count_{0};
  std::string reason_;
};

}  // namespace uda

#define UDA_CHECK(cond, msg)                                                        \
  do {                                                                              \
    if (!(cond))                                                                    \
      throw ::uda::UdaError(std::string(msg) + " (" __FILE__ ":" + std::to_string(__LINE__) + ")"); \
  } while (0)
