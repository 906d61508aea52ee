// Framed messages over node-local Unix stream sockets: the control channels between a reduce task's
// process and the node merge service, and between the provider front end and its node daemon.
//
// Frame: u32 type, u32 payload length, payload; one file descriptor may ride along (SCM_RIGHTS).
// Socket names: a path, or "@name" for the Linux abstract namespace (no file, so no stale socket files
// and no directory both sides must see; access is checked from the peer's credentials instead).
#pragma once
#include <sys/socket.h>
#include <sys/types.h>
#include <sys/un.h>

#include <cstdint>
#include <cstring>
#include <string>

namespace uda {
namespace frame {

constexpr uint32_t kMaxPayload = 64u << 20;

bool write_all(int fd, const void* p, size_t n);
bool send_msg(int sock, uint32_t type, const std::string& payload, int pass_fd = -1);
// false on EOF, error, an oversized frame or a receive timeout (SO_RCVTIMEO). *fd_out gets a passed
// descriptor (-1 if none).
bool recv_msg(int sock, uint32_t* type, std::string* payload, int* fd_out);

template <typename T>
void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <typename T>
T get(const std::string& s, size_t at) {
  T v{};
  if (at + sizeof(T) <= s.size()) std::memcpy(&v, s.data() + at, sizeof(T));
  return v;
}
// length-prefixed string
void put_str(std::string& s, const std::string& v);
// reads the string at *at and advances it; "" past the end
std::string get_str(const std::string& s, size_t* at);

// Poll `fd` for up to `us` microseconds before a blocking read (hand-overs that answer within tens of
// microseconds cost less than two scheduler wake-ups this way).
void spin_readable(int fd, int us);

// Address of a socket name ("@name": abstract namespace). Throws UdaError when the name does not fit.
sockaddr_un unix_addr(const std::string& name, socklen_t* len);
// Listening socket bound to `name` (a stale socket file is replaced; a path is made connectable by
// every local user: callers authenticate peers by their credentials). Throws UdaError.
int unix_listen(const std::string& name, int backlog);
// Connected socket, or -1 with errno set.
int unix_connect(const std::string& name);
// The connecting process's credentials (SO_PEERCRED).
bool peer_cred(int fd, uid_t* uid, pid_t* pid);

}  // namespace frame
}  // namespace uda
