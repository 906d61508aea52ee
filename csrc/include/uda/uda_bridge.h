/* UdaBridge C ABI: the host-facing API of libuda.so.
 *
 * Parity with the reference JNI surface (src/UdaBridge.cc, plugins/shared/com/mellanox/hadoop/
 * mapred/UdaBridge.java:49-145):
 *   entry points  startNative / doCommandNative / reduceExitMsgNative / setLogLevelNative
 *                 -> uda_start / uda_do_command / uda_reduce_exit / uda_set_log_level
 *   callbacks     fetchOverMessage, dataFromUda, getPathUda, getConfData, logToJava, failureInUda
 *                 -> uda_callbacks
 * Differences (MI355X-native design): the API is handle-based so one process can host a provider
 * and several consumers (tests, the single-node loopback config), and it is plain C so any host
 * (the JNI shim in csrc/bridge/jni_shim.cc, Python, a C++ driver) can drive it.
 *
 * Failure contract: any native failure after uda_start succeeds is reported exactly once through
 * callbacks.failure (the host then falls back to its vanilla shuffle, UdaShuffleConsumerPluginShared
 * .java:162-232); calls made on the host thread return a negative status instead of throwing.
 */
#ifndef UDA_BRIDGE_H_
#define UDA_BRIDGE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UDA_PATH_MAX 4096

/* IndexRecordBridge {startOffset, rawLength, partLength, pathMOF} (IndexRecordBridge.java:26-34). */
typedef struct uda_index_record {
  int64_t start_offset;
  int64_t raw_length;
  int64_t part_length;
  char path[UDA_PATH_MAX];
} uda_index_record;

typedef struct uda_callbacks {
  void* ctx;
  /* progress: called every PROGRESS_REPORT_LIMIT (20) fetched MOFs and at the end of fetching */
  void (*fetch_over)(void* ctx);
  /* merged data for the reducer: whole records, <= kv buffer size; return 0 to continue */
  int (*data_from_uda)(void* ctx, const void* buf, int32_t len);
  /* provider: resolve (job, map attempt, reduce) -> MOF index record; return 0 on success */
  int (*get_path)(void* ctx, const char* job_id, const char* map_id, int32_t reduce_id,
                  uda_index_record* out);
  /* configuration pull: write the value of `key` (or `dflt`) into out[0..outlen); return length */
  int (*get_conf)(void* ctx, const char* key, const char* dflt, char* out, int32_t outlen);
  /* log sink: severity 1=fatal .. 6=trace (UdaBridge.java:106-132) */
  void (*log)(void* ctx, const char* msg, int32_t severity);
  /* fatal native failure -> host falls back to vanilla shuffle */
  void (*failure)(void* ctx, const char* reason);
} uda_callbacks;

typedef struct uda_handle uda_handle;

/* Start a MOFSupplier (is_net_merger = 0) or a NetMerger (is_net_merger = 1). `argv` carries the
 * CLI options (-w -r -a -m -g -t -s). Returns NULL on failure (reason logged). */
uda_handle* uda_start(int is_net_merger, int argc, const char* const* argv, int log_level,
                      int log_to_file, const uda_callbacks* cb);
/* Java->native command "<n>:<id>:p1:..." (INIT/FETCH/FINAL/EXIT, C2JNexus.h:36-47). */
int uda_do_command(uda_handle* h, const char* cmd);
/* Reducer close: stop and join the merge, free everything (reduceExitMsgNative). */
int uda_reduce_exit(uda_handle* h);
/* Process-wide log threshold (setLogLevelNative). */
void uda_set_log_level(int level);
/* Release a handle after EXIT / reduce_exit. */
void uda_destroy(uda_handle* h);
/* Status string of the last failure on this handle ("" if none). */
const char* uda_last_error(uda_handle* h);
/* Version string (the reference logs "UDA version" for automation, MOFSupplierMain.cc:97-99). */
const char* uda_version(void);

/* Provider extension: register an in-memory MOF (host buffer) for (job, map); `index` holds
 * 3 int64 per reduce partition {start_offset, raw_length, part_length}. The data must outlive
 * the handle. Used by the loopback config and tests; real MOFs are resolved through get_path. */
int uda_provider_register_mof(uda_handle* h, const char* job_id, const char* map_id,
                              const void* data, int64_t len, const int64_t* index,
                              int32_t num_partitions);

/* Provider extension: register an HBM-resident MOF: `data` is device memory of HIP device `device`
 * (-1 = host memory, same as uda_provider_register_mof). Reducers on the GPU backend fetch a
 * descriptor of each partition (device address, or an IPC handle across processes) and merge it in
 * place; other reducers get the bytes through a device-to-host copy. */
int uda_provider_register_mof_device(uda_handle* h, const char* job_id, const char* map_id,
                                     const void* data, int64_t len, const int64_t* index,
                                     int32_t num_partitions, int32_t device);

/* Consumer/provider statistics as a JSON object (bytes fetched, GB/s, wait time, ...), written
 * NUL-terminated into out. Returns the length of the whole object (like snprintf): a result >= outlen
 * means it was cut and a buffer of result + 1 bytes holds it; -1 on a bad handle or buffer. */
int uda_stats_json(uda_handle* h, char* out, int32_t outlen);

#ifdef __cplusplus
}

#include <string>
#include <vector>
/* The whole statistics object, whatever its size ("{}" on a bad handle). */
inline std::string uda_stats_string(uda_handle* h) {
  std::vector<char> buf(8192);
  for (;;) {
    const int n = uda_stats_json(h, buf.data(), (int32_t)buf.size());
    if (n < 0) return "{}";
    if (n < (int)buf.size()) return std::string(buf.data(), (size_t)n);
    buf.resize((size_t)n + 1);
  }
}
#endif

#endif /* UDA_BRIDGE_H_ */
