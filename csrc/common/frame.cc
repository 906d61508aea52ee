// Framed Unix-socket messages. See uda/frame.h.
#include "uda/frame.h"

#include <poll.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>

#include "uda/error.h"

namespace uda {
namespace frame {

bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    c += w;
    n -= (size_t)w;
  }
  return true;
}

bool send_msg(int sock, uint32_t type, const std::string& payload, int pass_fd) {
  uint32_t hdr[2] = {type, (uint32_t)payload.size()};
  if (pass_fd < 0) {
    std::string buf(reinterpret_cast<const char*>(hdr), sizeof(hdr));
    buf += payload;
    return write_all(sock, buf.data(), buf.size());
  }
  msghdr mh{};
  iovec iov{hdr, sizeof(hdr)};
  mh.msg_iov = &iov;
  mh.msg_iovlen = 1;
  alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
  std::memset(cbuf, 0, sizeof(cbuf));
  mh.msg_control = cbuf;
  mh.msg_controllen = sizeof(cbuf);
  cmsghdr* cm = CMSG_FIRSTHDR(&mh);
  cm->cmsg_level = SOL_SOCKET;
  cm->cmsg_type = SCM_RIGHTS;
  cm->cmsg_len = CMSG_LEN(sizeof(int));
  std::memcpy(CMSG_DATA(cm), &pass_fd, sizeof(int));
  ssize_t w;
  do {
    w = ::sendmsg(sock, &mh, MSG_NOSIGNAL);
  } while (w < 0 && errno == EINTR);
  if (w <= 0) return false;
  if ((size_t)w < sizeof(hdr) && !write_all(sock, reinterpret_cast<char*>(hdr) + w, sizeof(hdr) - (size_t)w))
    return false;
  return write_all(sock, payload.data(), payload.size());
}

bool recv_msg(int sock, uint32_t* type, std::string* payload, int* fd_out) {
  uint32_t hdr[2];
  size_t got = 0;
  *fd_out = -1;
  while (got < sizeof(hdr)) {
    msghdr mh{};
    iovec iov{reinterpret_cast<char*>(hdr) + got, sizeof(hdr) - got};
    mh.msg_iov = &iov;
    mh.msg_iovlen = 1;
    alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
    mh.msg_control = cbuf;
    mh.msg_controllen = sizeof(cbuf);
    const ssize_t r = ::recvmsg(sock, &mh, MSG_CMSG_CLOEXEC);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    for (cmsghdr* cm = CMSG_FIRSTHDR(&mh); cm; cm = CMSG_NXTHDR(&mh, cm))
      if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) std::memcpy(fd_out, CMSG_DATA(cm), sizeof(int));
    got += (size_t)r;
  }
  *type = hdr[0];
  if (hdr[1] > kMaxPayload) return false;
  payload->resize(hdr[1]);
  got = 0;
  while (got < hdr[1]) {
    const ssize_t r = ::recv(sock, &(*payload)[got], hdr[1] - got, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    got += (size_t)r;
  }
  return true;
}

void put_str(std::string& s, const std::string& v) {
  put<uint32_t>(s, (uint32_t)v.size());
  s += v;
}

std::string get_str(const std::string& s, size_t* at) {
  const uint32_t n = get<uint32_t>(s, *at);
  if (*at + 4 + n > s.size()) {
    *at = s.size();
    return std::string();
  }
  std::string v = s.substr(*at + 4, n);
  *at += 4 + n;
  return v;
}

void spin_readable(int fd, int us) {
  pollfd pf{fd, POLLIN, 0};
  const auto t0 = std::chrono::steady_clock::now();
  while (::poll(&pf, 1, 0) == 0 && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(us)) {
  }
}

sockaddr_un unix_addr(const std::string& name, socklen_t* len) {
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  if (name.size() >= sizeof(a.sun_path) || name.empty()) throw UdaError("bad Unix socket name: '" + name + "'");
  if (name[0] == '@') {  // abstract: a leading NUL, the name's bytes, no terminator
    std::memcpy(a.sun_path + 1, name.data() + 1, name.size() - 1);
    *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + name.size());
  } else {
    std::memcpy(a.sun_path, name.c_str(), name.size() + 1);
    *len = (socklen_t)sizeof(a);
  }
  return a;
}

int unix_listen(const std::string& name, int backlog) {
  socklen_t len = 0;
  sockaddr_un a = unix_addr(name, &len);
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw UdaError(std::string("socket: ") + strerror(errno));
  if (name[0] != '@') ::unlink(name.c_str());
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), len) != 0 || ::listen(fd, backlog) != 0) {
    const std::string e = strerror(errno);
    ::close(fd);
    throw UdaError("cannot listen on " + name + ": " + e);
  }
  // a path gets the mode of the process's umask; peers are authenticated by SO_PEERCRED, so every local
  // user may connect (chmod after bind instead of a process-wide umask change: other threads of a JVM
  // host create files meanwhile)
  if (name[0] != '@') (void)::chmod(name.c_str(), 0666);
  return fd;
}

int unix_connect(const std::string& name) {
  socklen_t len = 0;
  sockaddr_un a;
  try {
    a = unix_addr(name, &len);
  } catch (const std::exception&) {
    errno = EINVAL;
    return -1;
  }
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), len) != 0) {
    const int e = errno;
    ::close(fd);
    errno = e;
    return -1;
  }
  return fd;
}

bool peer_cred(int fd, uid_t* uid, pid_t* pid) {
  ucred c{};
  socklen_t n = sizeof(c);
  if (::getsockopt(fd, SOL_SOCKET, SO_PEERCRED, &c, &n) != 0) return false;
  *uid = c.uid;
  *pid = c.pid;
  return true;
}

}  // namespace frame
}  // namespace uda
