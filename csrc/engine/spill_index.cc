// Hadoop map-output index files (SpillRecord). See uda/ifile.h.
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "uda/safe_file.h"
#include <stdexcept>

#include "uda/ifile.h"

namespace uda {

uint32_t crc32_ieee(const uint8_t* p, size_t n, uint32_t crc) {
  static uint32_t table[256];
  static const bool init = [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    return true;
  }();
  (void)init;
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

namespace {
void put_be64(uint8_t* d, int64_t v) {
  for (int i = 7; i >= 0; --i) {
    d[i] = (uint8_t)(v & 0xFF);
    v = (int64_t)((uint64_t)v >> 8);
  }
}
int64_t get_be64(const uint8_t* s) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | s[i];
  return (int64_t)v;
}
}  // namespace

void write_spill_index(const std::string& path, const std::vector<int64_t>& index) {
  std::vector<uint8_t> b(index.size() * 8 + 8);
  for (size_t i = 0; i < index.size(); ++i) put_be64(&b[i * 8], index[i]);
  put_be64(&b[index.size() * 8], (int64_t)crc32_ieee(b.data(), index.size() * 8));
  const int fd = create_private_file(path, O_WRONLY);
  if (fd < 0) throw std::runtime_error("cannot create " + path + ": " + strerror(errno));
  const bool ok = ::write(fd, b.data(), b.size()) == (ssize_t)b.size();
  ::close(fd);
  if (!ok) throw std::runtime_error("cannot write " + path);
}

bool read_spill_index(const std::string& path, std::vector<int64_t>* index, std::string* why) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (why) *why = "cannot open " + path + ": " + strerror(errno);
    return false;
  }
  std::vector<uint8_t> b;
  uint8_t chunk[65536];
  for (;;) {
    const ssize_t r = ::read(fd, chunk, sizeof(chunk));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    b.insert(b.end(), chunk, chunk + r);
  }
  ::close(fd);
  if (b.size() < 8 || (b.size() - 8) % 24 != 0) {
    if (why) *why = path + ": not a map output index (" + std::to_string(b.size()) + " bytes)";
    return false;
  }
  const size_t body = b.size() - 8;
  if ((uint32_t)get_be64(&b[body]) != crc32_ieee(b.data(), body)) {
    if (why) *why = path + ": index checksum mismatch";
    return false;
  }
  index->resize(body / 8);
  for (size_t i = 0; i < body / 8; ++i) (*index)[i] = get_be64(&b[i * 8]);
  return true;
}

}  // namespace uda
