// UDA_START_TRACE=1: one stderr line per step of a hosted reduce task's start (client connect, the front
// end's routing, the daemon's adoption and handshake, the session's READY), CLOCK_BOOTTIME ms, so the
// steps of one task line up across the three processes by its HELLO token. Off: one getenv, once.
#pragma once
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace uda {

inline void start_trace(const char* step, uint64_t token) {
  static const bool on = [] {
    const char* e = std::getenv("UDA_START_TRACE");
    return e && *e && *e != '0';
  }();
  if (!on) return;
  timespec ts{};
  clock_gettime(CLOCK_BOOTTIME, &ts);
  std::fprintf(stderr, "[start-trace] pid %d %.3f %s %016llx\n", (int)getpid(), (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6,
               step, (unsigned long long)token);
}

}  // namespace uda
