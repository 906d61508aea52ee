// UDA_STALL_PROBE=<seconds>: a diagnostic for stalls of one watched thread (the node daemon's control
// channel). Every 2 ms a sampler thread reads the watched thread's /proc state and syscall; once it has
// been out of its idle wait (asleep in recvmsg) for 6 ms, every thread of the process that is running,
// in uninterruptible sleep, ran >= 1 ms since the last sample, or is the watched one, is printed each 5 ms
// (name, state, CPU time and minor faults since the last sample, kernel wait channel, syscall and first
// arguments) until the watched thread is idle again. A sampler wake-up more than 20 ms late and each
// change of the cgroup's throttle count are printed too. The sampler allocates nothing once started (raw
// open/read/getdents64/write on stack buffers): a thread stuck on a malloc arena's lock or on the
// address-space lock never holds it up. Off: one getenv, once.
#pragma once
#include <fcntl.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "uda/thread_name.h"

namespace uda {

namespace stall_probe_detail {
inline std::atomic<int>& watched() {
  static std::atomic<int> t{0};
  return t;
}
// The file's first `cap - 1` bytes, trailing newlines and blanks cut; "" if unreadable.
inline const char* read_small(const char* path, char* buf, size_t cap) {
  buf[0] = 0;
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return buf;
  const ssize_t n = ::read(fd, buf, cap - 1);
  ::close(fd);
  size_t k = n > 0 ? (size_t)n : 0;
  while (k > 0 && (buf[k - 1] == '\n' || buf[k - 1] == ' ')) --k;
  buf[k] = 0;
  return buf;
}
inline const char* task_file(int tid, const char* leaf, char* buf, size_t cap) {
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/self/task/%d/%s", tid, leaf);
  return read_small(path, buf, cap);
}
inline char thread_state(int tid) {  // the field after "(comm)" in /proc/self/task/<tid>/stat
  char s[512];
  task_file(tid, "stat", s, sizeof(s));
  const char* p = std::strrchr(s, ')');
  return p && p[1] == ' ' && p[2] ? p[2] : '?';
}
inline const char* syscall_head(int tid, char* buf, size_t cap) {  // "<nr> <arg0> <arg1>" or "running"
  task_file(tid, "syscall", buf, cap);
  char* q = buf;
  for (int f = 0; f < 3 && q; ++f) q = std::strchr(q + 1, ' ');
  if (q) *q = 0;
  return buf;
}
inline double now_ms() {
  timespec ts{};
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec / 1e6;
}
template <typename... A>
inline void say(const char* fmt, A... a) {
  char line[640];
  const int n = std::snprintf(line, sizeof(line), fmt, a...);
  if (n > 0) (void)!::write(2, line, (size_t)std::min<int>(n, (int)sizeof(line) - 1));
}
struct Prev {  // per thread: CPU time and minor faults at the last sweep (open addressing by tid)
  int tid;
  unsigned long long run_ns, minflt;
};
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
    name_thread("uda-stall-probe");
    constexpr size_t kSlots = 1 << 14;
    std::vector<Prev> prev(kSlots, Prev{0, 0, 0});  // the sampler's only allocation
    const double end = now_ms() + dur_ms;
    double busy_since = -1, last_dump = -1, last_wake = now_ms();
    int lines = 0;
    const int pid = (int)getpid();
    char thr0[128] = "", cs[512], sc[128];
    unsigned long long on0 = 0, wait0 = 0;
    while (now_ms() < end && lines < 20000) {
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      const double tw = now_ms();
      {  // this sampler itself kept from running, and cgroup CPU throttling
        read_small("/sys/fs/cgroup/cpu.stat", cs, sizeof(cs));
        char thr[128] = "";
        if (const char* a = std::strstr(cs, "nr_throttled")) {
          size_t k = 0;
          while (a[k] && a[k] != '\n' && k + 1 < sizeof(thr)) thr[k] = a[k], ++k;
          thr[k] = 0;
        }
        // the sampler's own CPU time and run-queue wait (schedstat): a late wake-up spent runnable but
        // off the CPU (starved) shows as run-queue wait; stopped or blocked in the kernel shows as neither
        char ss[128];
        read_small("/proc/thread-self/schedstat", ss, sizeof(ss));
        char* e1 = nullptr;
        const unsigned long long on_ns = std::strtoull(ss, &e1, 10), wait_ns = std::strtoull(e1, nullptr, 10);
        if (tw - last_wake > 20 || std::strcmp(thr, thr0) != 0) {
          say("[stall-probe] pid %d %.3f sampler gap %.1f ms (on cpu %.1f ms, run-queue wait %.1f ms), %s\n", pid, tw,
              tw - last_wake, (double)(on_ns - on0) / 1e6, (double)(wait_ns - wait0) / 1e6, thr);
          ++lines;
        }
        on0 = on_ns;
        wait0 = wait_ns;
        std::memcpy(thr0, thr, sizeof(thr0));
        last_wake = tw;
      }
      const int w = watched().load();
      syscall_head(w, sc, sizeof(sc));
      // waiting for the next message: in recvmsg, asleep (not blocked in it on a lock or a fault: D)
      const bool idle = std::strncmp(sc, "47 ", 3) == 0 && thread_state(w) == 'S';
      const double t = now_ms();
      if (idle) {
        if (busy_since >= 0 && t - busy_since >= 6) say("[stall-probe] pid %d %.3f end busy %.1f ms\n", pid, t, t - busy_since);
        busy_since = -1;
        continue;
      }
      auto sweep = [&](bool print) {  // print: the threads that are running, blocked, or ran >= 1 ms since
        const int dfd = ::open("/proc/self/task", O_RDONLY | O_DIRECTORY | O_CLOEXEC);
        if (dfd < 0) return;
        alignas(8) char dents[8192];
        for (;;) {
          const long n = syscall(SYS_getdents64, dfd, dents, sizeof(dents));
          if (n <= 0) break;
          for (long off = 0; off < n;) {
            const unsigned short reclen = *reinterpret_cast<const unsigned short*>(dents + off + 16);
            const char* name = dents + off + 19;  // d_ino 8, d_off 8, d_reclen 2, d_type 1
            off += reclen;
            if (name[0] < '0' || name[0] > '9') continue;
            const int tid = std::atoi(name);
            char stat[512], sched[128], comm[32], wchan[64], tsc[128];
            task_file(tid, "stat", stat, sizeof(stat));
            const char* rp = std::strrchr(stat, ')');
            if (!rp || rp[1] != ' ' || !rp[2]) continue;
            const char st = rp[2];
            unsigned long long minflt = 0;  // the 8th field after the state
            {
              const char* q = rp + 2;
              for (int f = 0; f < 7 && q; ++f) q = std::strchr(q + 1, ' ');
              if (q) minflt = std::strtoull(q + 1, nullptr, 10);
            }
            const unsigned long long run_ns = std::strtoull(task_file(tid, "schedstat", sched, sizeof(sched)), nullptr, 10);
            size_t h = (size_t)tid * 2654435761u % kSlots, probes = 0;
            while (prev[h].tid != 0 && prev[h].tid != tid && ++probes < kSlots) h = (h + 1) % kSlots;
            if (probes >= kSlots) prev[h].tid = 0;  // full: reuse a slot
            Prev& pv = prev[h];
            const bool seen = pv.tid == tid;
            const double run_ms = seen ? (double)(run_ns - pv.run_ns) / 1e6 : 0.0;
            const unsigned long long flt = seen ? minflt - pv.minflt : 0;
            pv = Prev{tid, run_ns, minflt};
            if (!print || (tid != w && st != 'R' && st != 'D' && run_ms < 1.0)) continue;
            say("[stall-probe] pid %d %.3f busy %.1f tid %d%s %s %c ran %.1f ms faults %llu wchan %s sys %s\n", pid, t,
                t - busy_since, tid, tid == w ? "*" : "", task_file(tid, "comm", comm, sizeof(comm)), st, run_ms, flt,
                task_file(tid, "wchan", wchan, sizeof(wchan)), syscall_head(tid, tsc, sizeof(tsc)));
            ++lines;
          }
        }
        ::close(dfd);
      };
      if (busy_since < 0) {
        busy_since = t;
        sweep(false);  // the baseline of the episode's run times
      }
      if (t - busy_since < 6 || (last_dump >= 0 && t - last_dump < 5)) continue;
      last_dump = t;
      sweep(true);
    }
  }).detach();
}

}  // namespace uda
