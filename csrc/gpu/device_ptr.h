// HBM-resident map outputs shared with reducers: the "memory region + rkey" analogue of the
// reference's registered RDMA buffers (src/DataNet/RDMAComm.cc:67-154, rkey exchange in the
// connection private data, RDMAComm.h:35-39).
//
// A provider that registers a MOF living in device memory answers a descriptor fetch (RTS with a
// negative buffer length) with the partition's device address instead of its bytes. The descriptor
// travels in the ACK's path field, so both transports carry it unchanged:
//   hbm@<node id>@<device>@<pid>@<hex address>@<hex IPC handle or ->@<offset from the IPC base>
// A reducer in the same process uses the address directly (peer access enabled when the devices
// differ, so xGMI carries the reads); a reducer in another process on the node maps the
// provider's allocation with hipIpcOpenMemHandle (cached per handle) and adds the offset.
#pragma once
#include <cstdint>
#include <string>

namespace uda {
namespace gpu {

// IPC export of the allocation containing `ptr`: handle (hex) and the allocation base.
struct IpcExport {
  std::string handle_hex;  // "-" when the allocation cannot be shared across processes
  const uint8_t* base = nullptr;
  size_t size = 0;
  std::string refused;     // why no handle was exported (size in the hanging range), else empty
};
// Never throws; an allocation whose size lies in the hanging range (see ipc_safe_bytes) gets no
// handle ("-"), so reducers in other processes fetch its bytes instead of hanging in the import.
IpcExport ipc_export(const void* ptr);
bool ipc_size_ok(size_t bytes);
// Identity of this machine + boot (hex): descriptors are only mapped where it matches.
// Size to allocate for a block that other processes will map over hipIpc. On the ROCm 7 / dmabuf IPC
// path a block whose size modulo 2^32 lies in [2^31, 2^32) hangs the importing process in
// hipIpcOpenMemHandle or its first access (2.1 and 3.0 GiB hang, 1.9 and 4.2 GiB map fine;
// tools/ipc_size_probe.py, profiles/r2_ipc_size_probe.log), so such sizes are padded past the next
// multiple of 2^32.
const std::string& node_id();
size_t ipc_safe_bytes(size_t bytes);

// leased: the provider frees the allocation once every holder released it (its HBM store), so a
// reducer in another process closes its IPC mapping when it releases its last descriptor into it;
// registered MOFs (not leased) stay mapped for the process's life.
std::string make_device_descriptor(int device, const uint8_t* ptr, const IpcExport& ipc, bool leased = false);
bool is_device_descriptor(const std::string& s);
// Device address (usable on `my_device`) of a descriptor, or nullptr (reason in *why) when it cannot
// be used here: another node, no IPC handle, peer access impossible, import failure. Callers then
// fetch the partition's bytes.
const uint8_t* try_resolve_device_descriptor(const std::string& desc, int my_device, std::string* why);
// Same, throwing instead of returning nullptr.
const uint8_t* resolve_device_descriptor(const std::string& desc, int my_device);
// A resolved leased descriptor is done with: its IPC mapping is closed when no other descriptor of
// this process uses it.
void release_device_descriptor(const std::string& desc);
// Identity of a reducer that holds descriptors ("<node>:<pid>:<start ticks>:<task>"): the provider
// keeps what it hands out until this holder releases it, or its process is gone.
std::string reducer_holder_id(const std::string& task);
// IPC mappings this process holds open (tests).
int open_ipc_mappings();
// Device allocations freed by this process, by base address: an exporter that cached an allocation's
// IPC identity (IpcExchange) checks it before reusing the entry, since a new allocation can get the
// same address. alloc_epoch() numbers the frees; freed_since(base, e) is true if `base` was freed
// after epoch e.
uint64_t alloc_epoch();
void note_device_free(const void* base);
bool freed_since(const void* base, uint64_t epoch);
// Copy device memory at `src` (any device) to host `dst`.
void copy_device_to_host(void* dst, const void* src, int64_t bytes);

}  // namespace gpu
}  // namespace uda
