// Map-output store on local disks for jobs larger than HBM and pinned DRAM (the 4 TB tier).
//
// Reference counterparts: the provider's O_DIRECT libaio chunk reads of MOF files
// (DataEngine::aio_read_chunk_data, src/MOFServer/IndexInfo.cc:304-335, AIOHandler.cc:122-235) and
// the per-disk reader threads (src/AsyncIO/AsyncReaderManager.cc:16-49), plus the hybrid merge's
// spill files striped over the local dirs (src/Merger/MergeManager.cc:202-288).
//
// MI355X design: every MOF is one file, the files striped over the local dirs. A round's cells are
// staged disk -> pinned chunk ring (io_uring, O_DIRECT, 4 KiB-aligned supersets, a window of reads
// in flight) -> HBM (hipMemcpyAsync on the caller's stream, i.e. SDMA), chunks recycled once their
// H2D copy finished. HBM holds only the round slots, never the store.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "uda/aio.h"

namespace uda {
namespace gpu {

class DiskStore {
 public:
  DiskStore(int device, const std::vector<std::string>& dirs, const std::string& tag, int nfiles,
            int chunks = 8, int64_t chunk_bytes = 64ll << 20);
  ~DiskStore();  // closes and removes the files
  DiskStore(const DiskStore&) = delete;
  DiskStore& operator=(const DiskStore&) = delete;

  // Write `len` bytes of device memory as file `f` (padded to 4 KiB). Synchronous.
  void write_file(int f, const uint8_t* src_dev, int64_t len, hipStream_t s);

  struct Piece {
    int file;
    int64_t off;
    int64_t len;
    uint8_t* dst;  // device address
  };
  // Read every piece from disk and enqueue its H2D copy on `s`. Returns once all reads landed and
  // all copies are enqueued (the copies complete in stream order).
  void stage(const std::vector<Piece>& pieces, hipStream_t s);
  // Host copy of [off, off+len) of file f (tests / provider byte fetches).
  std::vector<uint8_t> read_host(int f, int64_t off, int64_t len);

  int64_t bytes_read() const { return bytes_read_; }
  int64_t bytes_written() const { return bytes_written_; }
  std::string describe() const;

 private:
  std::vector<std::string> paths_;
  std::vector<int> fds_;
  std::vector<int64_t> sizes_;  // padded file sizes
  std::unique_ptr<AsyncIO> aio_;
  int nchunks_;
  int64_t chunk_;
  uint8_t* ring_ = nullptr;
  std::vector<hipEvent_t> ev_;
  std::vector<bool> pending_;
  bool direct_ = true;
  int64_t bytes_read_ = 0, bytes_written_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace gpu
}  // namespace uda
