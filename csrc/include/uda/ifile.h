// IFile record streams, segments (sorted runs) and the CPU k-way merge.
//
// Parity map:
//   ifile_parse          <- BaseSegment::nextKVInternal (src/Merger/StreamRW.cc:334-404)
//   StreamSegment        <- Segment + KVOutput double buffer, switch_mem/join of a record split
//                           across two fetched chunks (StreamRW.cc:462-662)
//   MergeQueue           <- PriorityQueue / MergeQueue (src/Merger/MergeQueue.h:126-427)
//   write_kv_to_buffer   <- write_kv_to_stream (StreamRW.cc:151-225): greedy whole-record packing,
//                           EOF (-1,-1) appended to the last buffer when it fits
// The CPU engine is the correctness oracle and the in-house "reference algorithm" baseline.
#pragma once
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "uda/compare.h"
#include "uda/vint.h"

namespace uda {

struct RecordView {
  const uint8_t* key = nullptr;
  int32_t klen = 0;
  const uint8_t* val = nullptr;
  int32_t vlen = 0;
  int32_t hdr = 0;  // bytes of the two VInt headers
  int64_t size() const { return (int64_t)hdr + klen + vlen; }
};

enum class Parse { kRecord, kEof, kPartial, kCorrupt };

// Parse one record at [p, p+avail).
Parse ifile_parse(const uint8_t* p, size_t avail, RecordView* r);
int64_t ifile_record_size(int64_t klen, int64_t vlen);
void ifile_append(std::vector<uint8_t>* out, const uint8_t* k, int32_t kl, const uint8_t* v, int32_t vl);
void ifile_append_eof(std::vector<uint8_t>* out);
// Writes a record into buf (must have ifile_record_size bytes). Returns bytes written.
int64_t ifile_write(uint8_t* buf, const uint8_t* k, int32_t kl, const uint8_t* v, int32_t vl);

// ----------------------------------------------------------------------------- segments
// A sorted run of records. next() advances; cur() is valid after a true next().
class Segment {
 public:
  virtual ~Segment() = default;
  virtual bool next() = 0;  // false at EOF; throws UdaError on a corrupt stream
  const RecordView& cur() const { return cur_; }
  int index = 0;          // stable tie-break (fetch order / map order)
  int64_t records = 0;    // records produced so far
  KeyNorm norm{};         // normalized current key (first 16 content bytes), kept by MergeQueue
 protected:
  RecordView cur_;
};

// Whole stream in memory (owned or borrowed).
class MemorySegment : public Segment {
 public:
  MemorySegment(const uint8_t* data, size_t len) : p_(data), len_(len) {}
  MemorySegment(std::vector<uint8_t> owned)
      : owned_(std::move(owned)), p_(owned_.data()), len_(owned_.size()) {}
  bool next() override;

 private:
  std::vector<uint8_t> owned_;
  const uint8_t* p_;
  size_t len_;
  size_t pos_ = 0;
  bool eof_ = false;
};

// Pull-based chunk source: fills up to `cap` bytes at `dst`, returns bytes written, 0 at end.
// May block (network fetch, disk read, decompression).
using ChunkSource = std::function<int64_t(uint8_t* dst, int64_t cap)>;

// Stream consumed chunk by chunk through a two-buffer window; a record straddling the chunk
// boundary is joined into a carry buffer (the reference's switch_mem + join).
class StreamSegment : public Segment {
 public:
  StreamSegment(ChunkSource src, int64_t chunk_bytes);
  bool next() override;
  int64_t wait_ns() const { return wait_ns_; }  // time blocked in the source (total_wait_mem_time)

 private:
  bool refill();
  ChunkSource src_;
  std::vector<uint8_t> buf_;    // current chunk (with carried prefix in front)
  int64_t chunk_;
  size_t pos_ = 0, len_ = 0;
  bool src_done_ = false, eof_ = false;
  int64_t wait_ns_ = 0;
};

// ----------------------------------------------------------------------------- merge
class MergeQueue {
 public:
  explicit MergeQueue(KeyKind kind) : kind_(kind) {}
  // Takes ownership; primes the segment (empty segments are dropped).
  void insert(std::unique_ptr<Segment> s);
  // Advance to the next smallest record; false when all segments are exhausted.
  bool next();
  const RecordView& cur() const { return min_->cur(); }
  Segment* min_segment() const { return min_; }
  size_t size() const { return heap_.size(); }
  int64_t compares() const { return compares_; }

 private:
  bool less(const Segment* a, const Segment* b);
  void normalize(Segment* s);  // refresh the cached normalized key of the segment's current record
  void up(size_t i);
  void down(size_t i);
  KeyKind kind_;
  std::vector<std::unique_ptr<Segment>> heap_;
  Segment* min_ = nullptr;
  bool pending_advance_ = false;
  int64_t compares_ = 0;
};

// Greedy packing of merged records into caller buffers (write_kv_to_stream semantics): each
// buffer holds whole records; a record that does not fit stays pending for the next buffer; after
// the last record the EOF marker is appended if it fits, otherwise it goes alone into the next
// buffer. fill() returns true once the EOF marker has been written.
class KVWriter {
 public:
  explicit KVWriter(MergeQueue* q) : q_(q) {}
  bool fill(uint8_t* buf, int64_t cap, int64_t* len);
  int64_t records() const { return records_; }
  int64_t bytes() const { return bytes_; }

 private:
  MergeQueue* q_;
  bool pending_ = false;
  bool drained_ = false;
  int64_t records_ = 0, bytes_ = 0;
};

}  // namespace uda

namespace uda {

// ----------------------------------------------------------------------------- validation
// teravalidate for a merged reducer stream (reference: scripts/regression/mr-dstatExcel.sh:249-291
// runs Hadoop's TeraValidate on the job output). Buffers arrive as the host receives them
// (dataFromUda): whole records, the last buffer ending with the EOF marker. Checks the framing,
// the key order under the job's comparator, and accumulates the order-independent checksum
// (uda/hash.h) that is compared with the checksum of the map outputs.
class StreamValidator {
 public:
  explicit StreamValidator(KeyKind kind) : kind_(kind) {}
  void feed(const uint8_t* p, size_t n);
  int64_t records = 0;
  int64_t bytes = 0;           // record bytes (EOF excluded)
  int64_t buffers = 0;
  int64_t order_errors = 0;    // adjacent pairs out of order
  int64_t framing_errors = 0;  // partial record in a buffer, data after EOF, corrupt header
  uint64_t checksum = 0;
  bool eof = false;

 private:
  KeyKind kind_;
  std::string prev_key_;
  bool has_prev_ = false;
};

// Records and checksum of one IFile partition stream (stops at EOF or at the end of the bytes).
uint64_t ifile_checksum(const uint8_t* p, size_t n, int64_t* records, int64_t* bytes);


// A map output's index file (Hadoop SpillRecord, file.out.index): per partition three big-endian longs
// {startOffset, rawLength, partLength}, then the CRC32 of those bytes as a big-endian long. index holds
// 3 values per partition. The record getPathUda returns (IndexRecordBridge.java:26-34).
void write_spill_index(const std::string& path, const std::vector<int64_t>& index);
// false (why set) if the file is missing, short or fails its checksum
bool read_spill_index(const std::string& path, std::vector<int64_t>* index, std::string* why);
uint32_t crc32_ieee(const uint8_t* p, size_t n, uint32_t crc = 0);

}  // namespace uda
