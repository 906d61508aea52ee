// Leveled logger with a pluggable sink.
//
// Parity: reference `log()` macro + severities NONE..TRACE (src/include/IOUtility.h:151-195,
// src/CommUtils/IOUtility.cc:502-559). The numeric severities match the Java-side mapping in
// plugins/shared/com/mellanox/hadoop/mapred/UdaBridge.java:106-132 (1=fatal .. 6=trace), so a
// host bridge can route messages straight into its own logger (the `logToJava` callback).
#pragma once
#include <cstdarg>
#include <cstdint>
#include <string>

namespace uda {

enum Severity : int {
  kNone = 0,
  kFatal = 1,
  kError = 2,
  kWarn = 3,
  kInfo = 4,
  kDebug = 5,
  kTrace = 6,
};

using LogSink = void (*)(void* ctx, const char* msg, int severity);

// Process-wide threshold; messages with severity > threshold are dropped before formatting.
void log_set_threshold(int severity);
int log_threshold();
// Install a sink (nullptr restores the default stderr sink).
void log_set_sink(LogSink sink, void* ctx);
// Optional per-role file (reference: udaNetMerger.log / udaMOFSupplier.log, IOUtility.cc:406-466).
bool log_open_file(const std::string& dir, const std::string& role);
void log_close_file();

// Executables (never a library hosted by a JVM, which owns these signals): on SIGSEGV / SIGBUS / SIGILL /
// SIGFPE / SIGABRT write "<who> pid N: fatal signal S" and a raw backtrace to stderr, then die of the
// same signal. A process that dies silently (no exception text) otherwise leaves only "connection lost"
// at its peers.
void install_crash_reporter(const char* who);

void log_write(int severity, const char* file, int line, const char* func, const char* fmt, ...)
    __attribute__((format(printf, 5, 6)));

}  // namespace uda

#define UDA_LOG(sev, ...)                                                   \
  do {                                                                      \
    if ((sev) <= ::uda::log_threshold())                                    \
      ::uda::log_write((sev), __FILE__, __LINE__, __func__, __VA_ARGS__);   \
  } while (0)
