// Host-side stream validation (teravalidate) and checksums for the regression tools and tests.
#include "uda/hash.h"
#include "uda/ifile.h"

namespace uda {

void StreamValidator::feed(const uint8_t* p, size_t n) {
  buffers++;
  size_t pos = 0;
  if (eof && n) {
    framing_errors++;
    return;
  }
  while (pos < n) {
    RecordView rv;
    const Parse r = ifile_parse(p + pos, n - pos, &rv);
    if (r == Parse::kEof) {
      eof = true;
      if (pos + 2 != n) framing_errors++;  // bytes after the EOF marker
      return;
    }
    if (r != Parse::kRecord) {  // a record split across buffers or a corrupt header
      framing_errors++;
      return;
    }
    if (has_prev_ &&
        key_compare(kind_, reinterpret_cast<const uint8_t*>(prev_key_.data()), (int)prev_key_.size(), rv.key,
                    rv.klen) > 0)
      order_errors++;
    prev_key_.assign(reinterpret_cast<const char*>(rv.key), (size_t)rv.klen);
    has_prev_ = true;
    checksum += record_hash(p + pos, rv.size());
    records++;
    bytes += rv.size();
    pos += (size_t)rv.size();
  }
}

uint64_t ifile_checksum(const uint8_t* p, size_t n, int64_t* records, int64_t* bytes) {
  uint64_t ck = 0;
  int64_t recs = 0, b = 0;
  size_t pos = 0;
  while (pos < n) {
    RecordView rv;
    if (ifile_parse(p + pos, n - pos, &rv) != Parse::kRecord) break;
    ck += record_hash(p + pos, rv.size());
    recs++;
    b += rv.size();
    pos += (size_t)rv.size();
  }
  if (records) *records = recs;
  if (bytes) *bytes = b;
  return ck;
}

}  // namespace uda
