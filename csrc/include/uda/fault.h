// Fault injection (tests and chaos runs). UDA_FAULT_<SITE>=<n> makes the n-th event at that site
// fail; the count restarts whenever the variable's value changes. Sites:
//   FETCH         a fetch request (transport round) fails          -> consumer failure callback
//   AIO           an AsyncIO read/write completes with -EIO         -> provider/consumer failure
//   DEVICE_ALLOC  a device (HBM) allocation fails                   -> failure callback / error
//   HOST_ALLOC    the consumer's fetch-buffer pool allocation fails -> INIT error (UdaRuntimeException)
//   STORE_SETUP   a provider HBM store loader fails to start       -> its requests are declined (bytes)
// Reference analogue: none (the reference only has the fallback path itself); SURVEY.md §7.4.
// A thread can carry its own spec instead (FaultScope): a reduce task's mapred.uda.fault.inject, e.g.
// "DEVICE_ALLOC=1,FETCH=3", applies on its merge thread only, so one of several tasks hosted by the same
// process (the node daemon's merge service) can be made to fail while the others run on.
#pragma once
#include <string>

namespace uda {
bool fault_hit(const char* site);

class FaultScope {
 public:
  explicit FaultScope(const std::string& spec);  // "" = none (the environment applies)
  ~FaultScope();
  FaultScope(const FaultScope&) = delete;
  FaultScope& operator=(const FaultScope&) = delete;

 private:
  void* prev_;
};
}  // namespace uda
