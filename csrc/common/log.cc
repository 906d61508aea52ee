// Logger implementation: threshold, sink, optional per-role log file.
#include "uda/log.h"

#include <atomic>
#include <cstdio>
#include <cstring>
#include <csignal>
#include <ctime>
#include <execinfo.h>
#include <mutex>
#include <sys/time.h>
#include <unistd.h>

#include "uda/compare.h"
#include "uda/error.h"

namespace uda {

namespace {
std::atomic<int> g_threshold{kInfo};
std::mutex g_mu;
LogSink g_sink = nullptr;
void* g_sink_ctx = nullptr;
FILE* g_file = nullptr;

const char* sev_name(int s) {
  static const char* names[] = {"NONE", "FATAL", "ERROR", "WARN", "INFO", "DEBUG", "TRACE"};
  return (s >= 0 && s <= 6) ? names[s] : "?";
}
}  // namespace

namespace {
char g_who[64] = "uda";

void crash_handler(int sig) {
  char msg[160];
  const int n = std::snprintf(msg, sizeof(msg), "%s pid %d: fatal signal %d (%s)\n", g_who, (int)::getpid(), sig,
                              sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : sig == SIGABRT ? "SIGABRT"
                              : sig == SIGFPE ? "SIGFPE" : sig == SIGILL ? "SIGILL" : "?");
  if (n > 0) (void)!::write(2, msg, (size_t)n);
  void* frames[64];
  const int k = ::backtrace(frames, 64);
  ::backtrace_symbols_fd(frames, k, 2);
  std::signal(sig, SIG_DFL);  // SA_RESETHAND already did; re-raise with the default action
  ::raise(sig);
}
}  // namespace

void install_crash_reporter(const char* who) {
  std::snprintf(g_who, sizeof(g_who), "%s", who);
  void* warm[1];
  (void)::backtrace(warm, 1);  // loads libgcc's unwinder now, not inside the handler
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_handler = crash_handler;
  sa.sa_flags = SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT}) ::sigaction(sig, &sa, nullptr);
}

void log_set_threshold(int s) { g_threshold.store(s < 0 ? 0 : (s > kTrace ? kTrace : s)); }
int log_threshold() { return g_threshold.load(std::memory_order_relaxed); }

void log_set_sink(LogSink sink, void* ctx) {
  std::lock_guard<std::mutex> g(g_mu);
  g_sink = sink;
  g_sink_ctx = ctx;
}

bool log_open_file(const std::string& dir, const std::string& role) {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_file) fclose(g_file);
  std::string path = (dir.empty() ? std::string(".") : dir) + "/uda" + role + ".log";
  g_file = fopen(path.c_str(), "a");
  return g_file != nullptr;
}

void log_close_file() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_file) fclose(g_file);
  g_file = nullptr;
}

void log_write(int sev, const char* file, int line, const char* func, const char* fmt, ...) {
  char body[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(body, sizeof(body), fmt, ap);
  va_end(ap);
  const char* base = strrchr(file, '/');
  base = base ? base + 1 : file;
  char msg[2400];
  snprintf(msg, sizeof(msg), "%s:%d %s() %s", base, line, func, body);

  std::unique_lock<std::mutex> g(g_mu);
  if (g_file) {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    struct tm tmv;
    localtime_r(&tv.tv_sec, &tmv);
    char ts[64];
    strftime(ts, sizeof(ts), "%Y-%m-%d %H:%M:%S", &tmv);
    fprintf(g_file, "%s.%03d %-5s [tid %d] %s\n", ts, (int)(tv.tv_usec / 1000), sev_name(sev),
            (int)gettid(), msg);
    fflush(g_file);
    return;
  }
  if (g_sink) {
    // call the host sink (Java logToJava / Python) without holding the logger lock: it may log
    // or take its own locks
    const LogSink sink = g_sink;
    void* ctx = g_sink_ctx;
    g.unlock();
    sink(ctx, msg, sev);
    return;
  }
  fprintf(stderr, "[uda %s] %s\n", sev_name(sev), msg);
}

bool FailureLatch::report(const std::string& why) {
  count_.fetch_add(1);
  bool expected = false;
  if (!failed_.compare_exchange_strong(expected, true)) return false;
  reason_ = why;
  UDA_LOG(kError, "failure reported: %s", why.c_str());
  if (hook_) hook_(why);
  return true;
}

KeyKind key_kind_from_class(const char* n) {
  static const char* text[] = {"org.apache.hadoop.io.Text", nullptr};
  static const char* raw[] = {"org.apache.hadoop.io.BooleanWritable", "org.apache.hadoop.io.ByteWritable",
                              "org.apache.hadoop.io.ShortWritable", "org.apache.hadoop.io.IntWritable",
                              "org.apache.hadoop.io.LongWritable", nullptr};
  static const char* bytes[] = {"org.apache.hadoop.io.BytesWritable",
                                "org.apache.hadoop.hbase.io.ImmutableBytesWritable", nullptr};
  auto in = [n](const char** arr) {
    for (; *arr; ++arr)
      if (strcmp(n, *arr) == 0) return true;
    return false;
  };
  if (!n) return KeyKind::kUnsupported;
  if (in(text)) return KeyKind::kText;
  if (in(raw)) return KeyKind::kRaw;
  if (in(bytes)) return KeyKind::kBytes;
  return KeyKind::kUnsupported;
}

const char* key_kind_name(KeyKind k) {
  switch (k) {
    case KeyKind::kText: return "text";
    case KeyKind::kRaw: return "raw";
    case KeyKind::kBytes: return "bytes";
    default: return "unsupported";
  }
}

}  // namespace uda
