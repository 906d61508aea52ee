// UDA_STALL_PROBE=<seconds>: a diagnostic for stalls of one watched thread (the node daemon's control
// channel). Every 2 ms a sampler thread reads the watched thread's /proc state and syscall; once it has
// been out of its idle wait (asleep in recvmsg) for 6 ms, every thread of the process that is running,
// in uninterruptible sleep, ran >= 1 ms since the last sample, or is the watched one, is printed each 5 ms
// (name, state, CPU time and minor faults since the last sample, kernel wait channel, syscall and first
// arguments) until the watched thread is idle again. Off: one getenv, once.
#pragma once
#include <dirent.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>

#include "uda/thread_name.h"

namespace uda {

namespace stall_probe_detail {
inline std::atomic<int>& watched() {
  static std::atomic<int> t{0};
  return t;
}
inline std::string read_small(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return "";
  char buf[256];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  std::string s(buf);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}
inline char thread_state(int tid) {  // the field after "(comm)" in /proc/self/task/<tid>/stat
  const std::string s = read_small("/proc/self/task/" + std::to_string(tid) + "/stat");
  const size_t p = s.rfind(')');
  return p != std::string::npos && p + 2 < s.size() ? s[p + 2] : '?';
}
inline std::string syscall_head(int tid) {  // "<nr> <arg0> <arg1>" or "running"
  std::string s = read_small("/proc/self/task/" + std::to_string(tid) + "/syscall");
  size_t at = 0;
  for (int f = 0; f < 3 && at != std::string::npos; ++f) at = s.find(' ', at + 1);
  return at == std::string::npos ? s : s.substr(0, at);
}
inline double now_ms() {
  timespec ts{};
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6;
}
}  // namespace stall_probe_detail

// The calling thread becomes the watched one; the first call starts the sampler (when enabled).
inline void stall_probe_watch() {
  using namespace stall_probe_detail;
  static const double secs = [] {
    const char* e = std::getenv("UDA_STALL_PROBE");
    return e ? std::atof(e) : 0.0;
  }();
  if (secs <= 0) return;
  const int self = (int)syscall(SYS_gettid);
  if (watched().exchange(self) != 0) return;
  const double dur_ms = secs * 1e3;
  std::thread([dur_ms] {
    const double end = now_ms() + dur_ms;
    double busy_since = -1, last_dump = -1;
    int lines = 0;
    std::unordered_map<int, std::pair<unsigned long long, unsigned long long>> prev;  // tid -> run ns, faults
    name_thread("uda-stall-probe");
    const int pid = (int)getpid();
    while (now_ms() < end && lines < 20000) {
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      const int w = watched().load();
      const std::string sc = syscall_head(w);
      // waiting for the next message: in recvmsg, asleep (not blocked in it on a lock or a fault: D)
      const bool idle = sc.rfind("47 ", 0) == 0 && thread_state(w) == 'S';
      const double t = now_ms();
      if (idle) {
        if (busy_since >= 0 && t - busy_since >= 6)
          std::fprintf(stderr, "[stall-probe] pid %d %.3f end busy %.1f ms\n", pid, t, t - busy_since);
        busy_since = -1;
        continue;
      }
      auto sweep = [&](bool print) {  // print: the threads that are running, blocked, or ran >= 1 ms since
        DIR* d = opendir("/proc/self/task");
        if (!d) return;
        while (dirent* e = readdir(d)) {
          if (e->d_name[0] == '.') continue;
          const int tid = std::atoi(e->d_name);
          const std::string dir = "/proc/self/task/" + std::to_string(tid) + "/";
          const std::string stat = read_small(dir + "stat");
          const size_t rp = stat.rfind(')');
          if (rp == std::string::npos || rp + 2 >= stat.size()) continue;
          const char st = stat[rp + 2];
          unsigned long long minflt = 0;  // the 8th field after the state
          {
            const char* q = stat.c_str() + rp + 2;
            for (int f = 0; f < 7 && q; ++f) q = std::strchr(q + 1, ' ');
            if (q) minflt = std::strtoull(q + 1, nullptr, 10);
          }
          const unsigned long long run_ns = std::strtoull(read_small(dir + "schedstat").c_str(), nullptr, 10);
          auto& pv = prev[tid];
          const double run_ms = pv.first ? (double)(run_ns - pv.first) / 1e6 : 0.0;
          const unsigned long long flt = pv.first ? minflt - pv.second : 0;
          pv = {run_ns, minflt};
          if (!print || (tid != w && st != 'R' && st != 'D' && run_ms < 1.0)) continue;
          std::fprintf(stderr, "[stall-probe] pid %d %.3f busy %.1f tid %d%s %s %c ran %.1f ms faults %llu wchan %s sys %s\n", pid, t,
                       t - busy_since, tid, tid == w ? "*" : "", read_small(dir + "comm").c_str(), st, run_ms, flt,
                       read_small(dir + "wchan").c_str(), syscall_head(tid).c_str());
          ++lines;
        }
        closedir(d);
      };
      if (busy_since < 0) {
        busy_since = t;
        sweep(false);  // the baseline of the episode's run times
      }
      if (t - busy_since < 6 || (last_dump >= 0 && t - last_dump < 5)) continue;
      last_dump = t;
      {  // CPU-quota throttling of the process's cgroup (all threads stop until the period ends)
        std::string cs = read_small("/sys/fs/cgroup/cpu.stat");
        const size_t a = cs.find("nr_throttled");
        if (a != std::string::npos) {
          cs = cs.substr(a);
          for (char& c : cs) c = c == '\n' ? ' ' : c;
          std::fprintf(stderr, "[stall-probe] pid %d %.3f busy %.1f cgroup %s\n", pid, t, t - busy_since, cs.c_str());
        }
      }
      sweep(true);
    }
  }).detach();
}

}  // namespace uda
