// RTS / ACK string codecs (wire-compatible with the reference strings) and fault injection.
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "uda/fault.h"
#include "uda/transport.h"

namespace uda {

namespace {
std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t start = 0;
  for (;;) {
    size_t p = s.find(sep, start);
    if (p == std::string::npos) {
      out.push_back(s.substr(start));
      return out;
    }
    out.push_back(s.substr(start, p - start));
    start = p + 1;
  }
}
int64_t to_i64(const std::string& s) { return std::strtoll(s.c_str(), nullptr, 10); }
uint64_t to_u64(const std::string& s) { return std::strtoull(s.c_str(), nullptr, 10); }
}  // namespace

std::string format_rts(const FetchRequest& r, uint64_t remote_addr, uint64_t req_ptr) {
  return r.job_id + ":" + r.map_id + ":" + std::to_string(r.fetched) + ":" + std::to_string(r.reduce_id) +
         ":" + std::to_string(remote_addr) + ":" + std::to_string(req_ptr) + ":" +
         std::to_string(r.buf_len) + ":" + std::to_string(r.mof_offset) + ":" +
         (r.buf_len < 0 ? (r.holder.empty() ? std::string("?") : r.holder)
                        : (r.path.empty() ? std::string("?") : r.path)) +
         ":" + std::to_string(r.raw_len) + ":" +
         std::to_string(r.part_len);
}

bool parse_rts(const std::string& s, FetchRequest* r, uint64_t* remote_addr, uint64_t* req_ptr) {
  auto f = split(s, ':');
  if (f.size() < 11) return false;
  r->job_id = f[0];
  r->map_id = f[1];
  r->fetched = to_i64(f[2]);
  r->reduce_id = (int)to_i64(f[3]);
  if (remote_addr) *remote_addr = to_u64(f[4]);
  if (req_ptr) *req_ptr = to_u64(f[5]);
  r->buf_len = to_i64(f[6]);
  r->mof_offset = to_i64(f[7]);
  // path = fields 8 .. n-3 (a path may itself contain ':')
  std::string path = f[8];
  for (size_t i = 9; i + 2 < f.size(); ++i) path += ":" + f[i];
  r->path = (path == "?") ? std::string() : path;
  if (r->buf_len < 0) {  // descriptor fetch / release: the path field is the holder
    r->holder = r->path;
    r->path.clear();
  }
  r->raw_len = to_i64(f[f.size() - 2]);
  r->part_len = to_i64(f[f.size() - 1]);
  return true;
}

// An error ack keeps what the provider knows of the partition: a declined descriptor fetch
// (kNotDeviceResident) tells the reducer how many bytes to fetch instead, and where they are in which MOF
// file (a reducer on the provider's node may read them itself). E:status:raw:part:offset:pathlen:path:error
// (path by length, error last: both may contain ':').
std::string format_ack(const FetchAck& a) {
  if (a.status != 0)
    return "E:" + std::to_string(a.status) + ":" + std::to_string(a.raw_len) + ":" + std::to_string(a.part_len) + ":" +
           std::to_string(a.mof_offset) + ":" + std::to_string(a.path.size()) + ":" + a.path + ":" + a.error;
  return std::to_string(a.raw_len) + ":" + std::to_string(a.part_len) + ":" + std::to_string(a.sent) + ":" +
         std::to_string(a.mof_offset) + ":" + a.path + ":";
}

bool parse_ack(const std::string& s, FetchAck* a) {
  if (s.rfind("E:", 0) == 0) {
    int64_t v[5];
    size_t at = 2;
    for (int i = 0; i < 5; ++i) {  // status, raw, part, offset, path length
      const size_t c = s.find(':', at);
      if (c == std::string::npos) return false;
      v[i] = to_i64(s.substr(at, c - at));
      at = c + 1;
    }
    if (v[4] < 0 || at + (size_t)v[4] + 1 > s.size() || s[at + (size_t)v[4]] != ':') return false;
    a->status = v[0] == 0 ? -1 : (int)v[0];
    a->raw_len = v[1];
    a->part_len = v[2];
    a->mof_offset = v[3];
    a->path = s.substr(at, (size_t)v[4]);
    a->error = s.substr(at + (size_t)v[4] + 1);
    return true;
  }
  auto f = split(s, ':');
  if (f.size() < 5) return false;
  a->status = 0;
  a->raw_len = to_i64(f[0]);
  a->part_len = to_i64(f[1]);
  a->sent = to_i64(f[2]);
  a->mof_offset = to_i64(f[3]);
  std::string path = f[4];
  for (size_t i = 5; i + 1 < f.size(); ++i) path += ":" + f[i];
  a->path = path;
  return true;
}

// ------------------------------------------------------------------------- fault injection
bool fault_should_fail_fetch() { return fault_hit("FETCH"); }

}  // namespace uda
