// Where the MOFSupplier finds HBM copies of Hadoop-written map output files: the provider's HBM store,
// either in the provider's own process (gpu::MofCache) or in the node daemon (node_daemon.h), which
// the provider front end in the NodeManager reaches over a control socket.
//
// Reference: a fetch is answered from the chunk the DataEngine read from the MOF file
// (src/MOFServer/IndexInfo.cc:238-274); here a descriptor fetch of a file-backed MOF is answered with the
// partition's device address in the store, and the reducer merges it where it lies.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace uda {

class DeviceStore {
 public:
  // status 0: `desc` is the partition's device descriptor (gpu/device_ptr.h); kNotDeviceResident
  // (uda/transport.h): declined, the reducer fetches the bytes instead; any other negative status:
  // an error for the reducer, `desc` says what.
  using Done = std::function<void(int status, const std::string& desc)>;
  virtual ~DeviceStore() = default;
  // The partition [offset, offset + len) of MOF file `path` of `job` as a descriptor holding a
  // reference of `holder` (released by release / release_holder). Loads the file on first touch and
  // calls done once the partition's bytes are in HBM (inline if they already are). false (*why set,
  // done never called) when the store declines at once.
  virtual bool acquire(const std::string& job, const std::string& path, const std::string& holder, int64_t offset,
                       int64_t len, Done done, std::string* why) = 0;
  virtual void release(const std::string& path, const std::string& holder) = 0;
  // every reference of `holder` on the job's MOFs ("*": on any job's)
  virtual void release_holder(const std::string& job, const std::string& holder) = 0;
  virtual void job_over(const std::string& job) = 0;
  virtual std::string stats_json() = 0;
};

struct LocalStoreOptions {
  int64_t capacity = 0;  // bytes over all devices
  std::vector<int> devices{0};
  double lease_s = 600;
  double idle_evict_s = 0;  // gpu::MofCache::Options::idle_evict_s
  bool cached_read = true;  // gpu::MofCache::Options::cached_read
};
// The store in this process (gpu/mof_cache.h).
std::unique_ptr<DeviceStore> make_local_device_store(const LocalStoreOptions& o);

}  // namespace uda
