// Command protocol parser/formatter. See uda/cmd.h for the reference mapping.
#include "uda/cmd.h"

#include <cstdlib>
#include <sstream>

namespace uda {

bool parse_cmd(const std::string& s, HadoopCmd* out) {
  out->params.clear();
  if (s.empty()) {  // C2JNexus.cc: an empty command is EXIT
    out->count = 1;
    out->header = kExitMsg;
    return true;
  }
  // count and header must be decimal numbers and the header a known command id (the reference's
  // atoi would turn a garbled header into EXIT)
  auto number = [](const std::string& t, int* v) {
    if (t.empty() || t.size() > 9) return false;
    for (char c : t)
      if (c < '0' || c > '9') return false;
    *v = std::atoi(t.c_str());
    return true;
  };
  size_t p = s.find(':');
  if (p == std::string::npos) return false;
  int count = 0, header = 0;
  if (!number(s.substr(0, p), &count)) return false;
  out->count = count;
  size_t start = p + 1;
  size_t end = s.find(':', start);
  if (!number(s.substr(start, end == std::string::npos ? std::string::npos : end - start), &header) ||
      header > (int)kRtLaunched)
    return false;
  out->header = (CmdId)header;
  if (end == std::string::npos) return true;
  start = end + 1;
  // count-1 params; all but the last are ':'-terminated, the last takes the remainder.
  for (int i = 0; i < out->count - 2; ++i) {
    end = s.find(':', start);
    if (end == std::string::npos) return false;
    out->params.push_back(s.substr(start, end - start));
    start = end + 1;
  }
  if (out->count >= 2) out->params.push_back(s.substr(start));
  return true;
}

std::string form_cmd(int id, const std::vector<std::string>& params) {
  std::string r = std::to_string(params.size() + 1) + ":" + std::to_string(id);
  for (const auto& p : params) {
    r += ':';
    r += p;
  }
  return r;
}

bool parse_options(const std::vector<std::string>& args, NetlevOptions* o, std::string* err) {
  for (size_t i = 0; i < args.size(); ++i) {
    const std::string& a = args[i];
    if (a.size() != 2 || a[0] != '-') {
      if (err) *err += "ignoring argument '" + a + "'; ";
      continue;
    }
    if (i + 1 >= args.size()) {
      if (err) *err += "missing value for " + a + "; ";
      return false;
    }
    const std::string& v = args[++i];
    switch (a[1]) {
      case 'w': o->wqes_per_conn = std::atoi(v.c_str()); break;
      case 'r': o->data_port = std::atoi(v.c_str()); break;
      case 'a': o->online = std::atoi(v.c_str()); break;
      case 'm': o->mode = std::atoi(v.c_str()); break;
      case 'g': o->log_dir = v; break;
      case 't': o->trace_level = std::atoi(v.c_str()); break;
      case 's': {
        int64_t kb = std::atoll(v.c_str());
        int64_t bytes = kb * 1024;
        bytes -= bytes % 4096;  // page aligned, C2JNexus.cc:105-119
        if (bytes <= 0) bytes = 4096;
        o->buf_size = bytes;
        break;
      }
      default:
        if (err) *err += "unknown option " + a + "; ";
        break;
    }
  }
  return true;
}

bool parse_init_params(const HadoopCmd& c, InitParams* p, std::string* err) {
  const auto& v = c.params;
  if (v.size() < 11) {
    if (err) *err = "INIT needs >= 11 params, got " + std::to_string(v.size());
    return false;
  }
  p->num_maps = std::atoi(v[0].c_str());
  p->job_id = v[1];
  p->reduce_task_id = v[2];
  p->lpq_size = std::atoi(v[3].c_str());
  p->max_buf_bytes = std::atoll(v[4].c_str());
  p->min_buf_bytes = std::atoll(v[5].c_str());
  p->key_class = v[6];
  p->codec = (v[7] == "null") ? std::string() : v[7];
  p->comp_block_size = std::atoll(v[8].c_str());
  p->shuffle_mem_bytes = std::atoll(v[9].c_str());
  int ndirs = std::atoi(v[10].c_str());
  p->local_dirs.clear();
  for (int i = 0; i < ndirs; ++i) {
    if (11 + (size_t)i >= v.size()) {
      if (err) *err = "INIT declares " + std::to_string(ndirs) + " dirs but carries fewer";
      return false;
    }
    p->local_dirs.push_back(v[11 + i]);
  }
  return true;
}

std::vector<std::string> init_params_to_strings(const InitParams& p) {
  std::vector<std::string> v = {std::to_string(p.num_maps),
                                p.job_id,
                                p.reduce_task_id,
                                std::to_string(p.lpq_size),
                                std::to_string(p.max_buf_bytes),
                                std::to_string(p.min_buf_bytes),
                                p.key_class,
                                p.codec.empty() ? "null" : p.codec,
                                std::to_string(p.comp_block_size),
                                std::to_string(p.shuffle_mem_bytes),
                                std::to_string(p.local_dirs.size())};
  for (const auto& d : p.local_dirs) v.push_back(d);
  return v;
}

bool parse_fetch_params(const HadoopCmd& c, FetchParams* f, std::string* err) {
  if (c.params.size() < 4) {
    if (err) *err = "FETCH needs 4 params";
    return false;
  }
  f->host = c.params[0];
  f->job_id = c.params[1];
  f->map_id = c.params[2];
  f->reduce_id = std::atoi(c.params[3].c_str());
  return true;
}

}  // namespace uda
