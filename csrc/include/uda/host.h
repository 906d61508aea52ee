// Host callback wrapper + configuration pull.
//
// Parity: UdaBridge_invoke_*_callback helpers (src/UdaBridge.cc:338-452) and the two config
// channels of the reference (SURVEY.md §5 "Config / flag system"): CLI options (-w -r -a -m -g -t
// -s, see uda/cmd.h) and `getConfData(key, default)` pulled from the host's JobConf. Environment
// variables UDA_CONF_<key with '.' -> '_'> override the host's answer (benchmarking knobs).
#pragma once
#include <cstdint>
#include <mutex>
#include <string>

#include "uda/error.h"
#include "uda/uda_bridge.h"

namespace uda {

struct IndexRec {
  int64_t start_offset = 0;
  int64_t raw_length = 0;
  int64_t part_length = 0;
  std::string path;
};

class Host {
 public:
  explicit Host(const uda_callbacks* cb);
  void fetch_over();
  int data_from_uda(const uint8_t* buf, int32_t len);
  bool get_path(const std::string& job, const std::string& map, int reduce, IndexRec* out);
  std::string get_conf(const std::string& key, const std::string& dflt);
  int64_t conf_i64(const std::string& key, int64_t dflt);
  double conf_f64(const std::string& key, double dflt);
  bool conf_bool(const std::string& key, bool dflt);
  // Report a fatal native failure once (-> failureInUda).
  void fail(const std::string& reason) { latch_.report(reason); }
  bool failed() const { return latch_.failed(); }
  const std::string& failure_reason() const { return latch_.first_reason(); }
  int failure_reports() const { return latch_.count(); }
  const uda_callbacks& raw() const { return cb_; }

 private:
  uda_callbacks cb_;
  FailureLatch latch_;
};

}  // namespace uda
