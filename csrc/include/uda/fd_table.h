// Grows the process's descriptor table to `want` slots (capped by RLIMIT_NOFILE, whose soft limit is
// raised to the hard one) while the process is still single-threaded. The kernel grows the table by
// doubling, and in a multi-threaded process each doubling waits for an RCU grace period while every
// other thread that opens a descriptor (a socket, a file, a memfd, a dma-buf) waits for it: on the GPU
// boxes that froze the node daemon for 90-180 ms at the start of its first wave of hosted tasks (threads
// in expand_files / __wait_rcu_gp, profiles/r6/r7_first_wave_stall.md). Tables never shrink, so growing it
// once up front removes those waits. Returns the table size reached (0: not grown).
#pragma once
#include <fcntl.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>

namespace uda {

inline int pregrow_fd_table(int want = 1 << 17) {
  rlimit rl{};
  if (::getrlimit(RLIMIT_NOFILE, &rl) != 0) return 0;
  if (rl.rlim_cur < rl.rlim_max) {
    rlimit up = rl;
    up.rlim_cur = rl.rlim_max;
    if (::setrlimit(RLIMIT_NOFILE, &up) == 0) rl = up;
  }
  const long top = (long)std::min<rlim_t>(rl.rlim_cur, (rlim_t)want) - 1;
  if (top < 64) return 0;
  const int base = ::open("/dev/null", O_RDONLY | O_CLOEXEC);
  if (base < 0) return 0;
  const int hi = ::fcntl(base, F_DUPFD_CLOEXEC, (int)top);  // the lowest free descriptor >= top
  ::close(base);
  if (hi < 0) return 0;
  ::close(hi);
  return (int)top + 1;
}

}  // namespace uda
