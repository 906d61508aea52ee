// Files a reduce task creates, appends to and reads back in its local directories (LPQ spills, their
// indexes, the checkpoint manifest). The directories may be writable by the job's user (YARN's
// usercache/<user>/appcache/...) while the task runs as another user (a node merge-service session), so
// nothing here follows a symlink planted at the name, and an existing file is only appended to or trusted
// when this process's user owns it.
#pragma once
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <string>

namespace uda {

// A fresh file at `path` (whatever was there is unlinked first; a name re-created in between fails
// with EEXIST instead of being followed). flags: O_WRONLY or O_RDWR.
inline int create_private_file(const std::string& path, int flags) {
  (void)::unlink(path.c_str());
  return ::open(path.c_str(), flags | O_CREAT | O_EXCL | O_NOFOLLOW | O_CLOEXEC, 0600);
}

// True if `path` is a regular file (not a symlink) owned by this process's effective user.
inline bool owned_regular_file(const std::string& path, struct stat* out = nullptr) {
  struct stat sb;
  if (::lstat(path.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_uid != ::geteuid()) return false;
  if (out) *out = sb;
  return true;
}

// Append-only descriptor of a file this process's user owns (created if missing); -1 (errno EPERM) for
// a symlink or somebody else's file.
inline int open_owned_append(const std::string& path) {
  const int fd = ::open(path.c_str(), O_WRONLY | O_APPEND | O_CREAT | O_NOFOLLOW | O_CLOEXEC, 0600);
  if (fd < 0) return -1;
  struct stat sb;
  if (::fstat(fd, &sb) != 0 || !S_ISREG(sb.st_mode) || sb.st_uid != ::geteuid()) {
    ::close(fd);
    errno = EPERM;
    return -1;
  }
  return fd;
}

inline bool write_all(int fd, const void* data, size_t len) {
  const char* p = static_cast<const char*>(data);
  while (len > 0) {
    const ssize_t n = ::write(fd, p, len);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) return false;
    p += n;
    len -= (size_t)n;
  }
  return true;
}

// Append one line to an owned file (the LPQ manifest).
inline bool append_owned_line(const std::string& path, const std::string& line) {
  const int fd = open_owned_append(path);
  if (fd < 0) return false;
  const std::string l = line + "\n";
  const bool ok = write_all(fd, l.data(), l.size());
  ::close(fd);
  return ok;
}

}  // namespace uda
