#include "uda/host.h"

#include <cstdlib>
#include <cstring>
#include <vector>

#include "uda/log.h"

namespace uda {

Host::Host(const uda_callbacks* cb) {
  std::memset(&cb_, 0, sizeof(cb_));
  if (cb) cb_ = *cb;
  latch_.set_hook([this](const std::string& why) {
    if (cb_.failure) cb_.failure(cb_.ctx, why.c_str());
  });
}

void Host::fetch_over() {
  if (cb_.fetch_over) cb_.fetch_over(cb_.ctx);
}

int Host::data_from_uda(const uint8_t* buf, int32_t len) {
  if (!cb_.data_from_uda) return 0;
  return cb_.data_from_uda(cb_.ctx, buf, len);
}

bool Host::get_path(const std::string& job, const std::string& map, int reduce, IndexRec* out) {
  if (!cb_.get_path) return false;
  uda_index_record r;
  std::memset(&r, 0, sizeof(r));
  if (cb_.get_path(cb_.ctx, job.c_str(), map.c_str(), reduce, &r) != 0) return false;
  out->start_offset = r.start_offset;
  out->raw_length = r.raw_length;
  out->part_length = r.part_length;
  r.path[UDA_PATH_MAX - 1] = 0;
  out->path = r.path;
  return true;
}

std::string Host::get_conf(const std::string& key, const std::string& dflt) {
  std::string env = "UDA_CONF_" + key;
  for (auto& c : env)
    if (c == '.' || c == '-') c = '_';
  if (const char* e = std::getenv(env.c_str())) return e;
  if (!cb_.get_conf) return dflt;
  std::vector<char> buf(4096);
  int n = cb_.get_conf(cb_.ctx, key.c_str(), dflt.c_str(), buf.data(), (int32_t)buf.size());
  if (n < 0) return dflt;
  if (n >= (int)buf.size()) n = (int)buf.size() - 1;
  return std::string(buf.data(), (size_t)n);
}

int64_t Host::conf_i64(const std::string& key, int64_t dflt) {
  std::string v = get_conf(key, std::to_string(dflt));
  if (v.empty()) return dflt;
  return std::strtoll(v.c_str(), nullptr, 10);
}

double Host::conf_f64(const std::string& key, double dflt) {
  std::string v = get_conf(key, std::to_string(dflt));
  if (v.empty()) return dflt;
  return std::atof(v.c_str());
}

bool Host::conf_bool(const std::string& key, bool dflt) {
  std::string v = get_conf(key, dflt ? "true" : "false");
  return v == "true" || v == "1" || v == "yes";
}

}  // namespace uda
