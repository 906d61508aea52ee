// Java <-> native command protocol and the native CLI option set.
//
// Parity: the command string format "<count>:<header>:p1:...:p(count-1)" where count includes the
// header (Java side: UdaCmd.formCmd, plugins/shared/com/mellanox/hadoop/mapred/UdaPlugin.java:577-586;
// native side: parse_hadoop_cmd, src/CommUtils/C2JNexus.cc:152-207). Command ids from
// src/include/C2JNexus.h:36-47. The last parameter may itself contain ':' (the reference parser
// takes the remainder verbatim), which matters for paths.
//
// CLI options (getopt -w -r -a -m -g -t -s; C2JNexus.cc:43-137): -s is given in KB and converted
// to bytes, rounded down to a 4 KiB multiple.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace uda {

enum CmdId : int {
  kExitMsg = 0,
  kNewMapMsg = 1,
  kFinalMsg = 2,
  kResult = 3,
  kFetchMsg = 4,
  kFetchOverMsg = 5,
  kJobOverMsg = 6,
  kInitMsg = 7,
  kMoreMsg = 8,
  kRtLaunched = 9,
};

struct HadoopCmd {
  int count = 1;              // header + params
  CmdId header = kExitMsg;
  std::vector<std::string> params;
};

// Parse a command string. Empty string == EXIT (reference behaviour). Returns false on a
// malformed string (missing separators for the declared count).
bool parse_cmd(const std::string& s, HadoopCmd* out);
// Format like UdaCmd.formCmd.
std::string form_cmd(int id, const std::vector<std::string>& params);

struct NetlevOptions {
  int wqes_per_conn = 256;   // -w
  int data_port = 9011;      // -r
  int online = 1;            // -a : merge approach (1 online, 2 hybrid, 0 = no-op in reference)
  int mode = 1;              // -m : 1 INTEGRATED, 0 STANDALONE
  std::string log_dir;       // -g
  int trace_level = -1;      // -t
  int64_t buf_size = 1024 * 1024;  // -s (KB on the command line)
};

// Parse argv-style options. Unknown options are reported and ignored (reference prints usage).
bool parse_options(const std::vector<std::string>& args, NetlevOptions* out, std::string* err);

// INIT message parameters (UdaPlugin.java:269-312 / reducer.cc:58-98).
struct InitParams {
  int num_maps = 0;
  std::string job_id;
  std::string reduce_task_id;
  int lpq_size = 0;
  int64_t max_buf_bytes = 1024 * 1024;
  int64_t min_buf_bytes = 16 * 1024;
  std::string key_class;
  std::string codec;        // empty when the Java side sent "null"
  int64_t comp_block_size = 256 * 1024;
  int64_t shuffle_mem_bytes = 0;
  std::vector<std::string> local_dirs;
};
bool parse_init_params(const HadoopCmd& cmd, InitParams* out, std::string* err);
std::vector<std::string> init_params_to_strings(const InitParams& p);

// FETCH parameters: host, jobId, mapAttemptId, reducePartition (UdaPlugin.java:324-331).
struct FetchParams {
  std::string host;
  std::string job_id;
  std::string map_id;
  int reduce_id = 0;
};
bool parse_fetch_params(const HadoopCmd& cmd, FetchParams* out, std::string* err);

}  // namespace uda
