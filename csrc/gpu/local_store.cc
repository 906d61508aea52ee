// DeviceStore over the HBM store of this process (provider/device_store.h, gpu/mof_cache.h).
#include <unistd.h>

#include <cstdlib>
#include <memory>
#include <string>

#include "uda/start_trace.h"
#include "../provider/device_store.h"
#include "device_ptr.h"
#include "mof_cache.h"
#include "uda/transport.h"

namespace uda {

namespace {

// the pid field of a reducer holder id (node:pid:start:task); -1 for any other form
int holder_pid(const std::string& holder) {
  const size_t a = holder.find(':');
  if (a == std::string::npos) return -1;
  const size_t b = holder.find(':', a + 1);
  if (b == std::string::npos) return -1;
  const std::string p = holder.substr(a + 1, b - a - 1);
  if (p.empty() || p.find_first_not_of("0123456789") != std::string::npos) return -1;
  return std::atoi(p.c_str());
}

class LocalDeviceStore : public DeviceStore {
 public:
  explicit LocalDeviceStore(const LocalStoreOptions& o) {
    gpu::MofCache::Options co;
    co.capacity = o.capacity;
    co.devices = o.devices;
    co.odirect = true;
    co.lease_s = o.lease_s;
    co.idle_evict_s = o.idle_evict_s;
    co.cached_read = o.cached_read;
    cache_ = std::make_unique<gpu::MofCache>(co);
    cache_->start_loaders();  // the loaders come up now, not under the first wave
  }

  bool acquire(const std::string& job, const std::string& path, const std::string& holder, int64_t offset,
               int64_t len, Done done, std::string* why) override {
    const int64_t need = offset + len;
    // a holder in this process (node:pid:start:task, gpu::reducer_holder_id) reads the HBM directly;
    // any other process maps it through the entry's hipIpc export, made on its first such fetch
    const bool local = holder_pid(holder) == (int)getpid() && holder.compare(0, holder.find(':'), gpu::node_id()) == 0;
    gpu::MofCache* cache = cache_.get();
    return cache_->acquire_async(
        job, path, holder, need,
        [done, offset, need, path, local, cache](bool ok, const gpu::MofCache::Ref& ref, const std::string& w) {
          if (!ok) return done(kNotDeviceResident, "provider HBM store: " + w);
          if (need > ref.len) return done(-4, "index beyond MOF file " + path);
          if (local || ref.ipc.handle_hex != "-")
            return done(0, gpu::make_device_descriptor(ref.device, ref.data + offset, ref.ipc, /*leased=*/true));
          start_trace("store_export_begin", 0);
          gpu::IpcExport x = cache->export_of(path);
          start_trace("store_export_end", 0);
          if (x.handle_hex == "-") x.base = ref.ipc.base;  // not exportable: the descriptor says so
          done(0, gpu::make_device_descriptor(ref.device, ref.data + offset, x, /*leased=*/true));
        },
        why);
  }
  void release(const std::string& path, const std::string& holder) override { cache_->release(path, holder); }
  void release_holder(const std::string& job, const std::string& holder) override {
    cache_->release_holder(job, holder);
  }
  void job_over(const std::string& job) override { cache_->job_over(job); }
  std::string stats_json() override {
    const gpu::MofCache::Stats st = cache_->stats();
    return "{\"loads\":" + std::to_string(st.loads) + ",\"hits\":" + std::to_string(st.hits) +
           ",\"holders\":" + std::to_string(st.holders) + ",\"releases\":" + std::to_string(st.releases) +
           ",\"holders_reaped\":" + std::to_string(st.holders_reaped) + ",\"load_wall_ms\":" +
           std::to_string(st.load_wall_ms) + ",\"open_ms\":" + std::to_string(st.open_ms) +
           ",\"open_alloc_ms\":" + std::to_string(st.open_alloc_ms) + ",\"open_export_ms\":" +
           std::to_string(st.open_export_ms) + ",\"open_file_ms\":" + std::to_string(st.open_file_ms) +
           ",\"open_file_max_ms\":" + std::to_string(st.open_file_max_ms) + ",\"load_gbps\":" +
           std::to_string(st.load_wall_ms > 0 ? (double)st.bytes_loaded / st.load_wall_ms / 1e6 : 0.0) +
           ",\"declined\":" + std::to_string(st.declined) + ",\"evictions\":" + std::to_string(st.evictions) +
           ",\"cached_reads\":" + std::to_string(st.cached_reads) +
           ",\"bytes_loaded\":" + std::to_string(st.bytes_loaded) + ",\"resident_bytes\":" +
           std::to_string(st.resident_bytes) + ",\"capacity\":" + std::to_string(cache_->capacity()) +
           ",\"load_ms\":" + std::to_string(st.load_ms) + ",\"first_miss_boot_ms\":" +
           std::to_string(st.first_miss_boot_ms) + ",\"first_read_boot_ms\":" + std::to_string(st.first_read_boot_ms) +
           ",\"last_landed_boot_ms\":" + std::to_string(st.last_landed_boot_ms) + "}";
  }

 private:
  std::unique_ptr<gpu::MofCache> cache_;
};

}  // namespace

std::unique_ptr<DeviceStore> make_local_device_store(const LocalStoreOptions& o) {
  return std::make_unique<LocalDeviceStore>(o);
}

}  // namespace uda
