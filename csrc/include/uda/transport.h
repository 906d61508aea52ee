// Shuffle transport: the fetch protocol between a reducer (NetMerger) and a map-output provider
// (MOFSupplier), independent of the wire.
//
// Parity: the reference's RDMA data path: the client posts an RTS
//   "job:map:fetched:reduce:remoteAddr:reqPtr:bufLen:mofOffset:mofPath:rawLen:partLen"
// (src/DataNet/RDMAClient.cc:559-600); the server RDMA-WRITEs min(chunk, bufLen) bytes of the
// partition and SENDs an ACK "rawLength:partLength:sent:offset:path:" (RDMAServer.cc:537-631).
// Credits bound in-flight requests per connection (wqes_per_conn, RDMAComm.cc:707-752).
//
// Backends here: `loopback` (in-process, zero-copy into the client buffer: the RDMA-WRITE
// analogue) and `tcp` (sockets, the same RTS/ACK strings inside a 16-byte netlev header, for
// multi-process / multi-host runs). The GPU data plane does not use this interface: partitions
// move HBM->HBM through RCCL all-to-all rounds (csrc/gpu/device_engine.cc).
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>

namespace uda {

struct FetchRequest {
  std::string job_id;
  std::string map_id;
  int reduce_id = 0;
  int64_t fetched = 0;   // bytes of the partition already received
  int64_t buf_len = 0;   // client buffer capacity
  // echoed back by the provider after the first chunk (saves re-resolving the index)
  int64_t mof_offset = -1;
  int64_t raw_len = -1;
  int64_t part_len = -1;
  std::string path;
  // descriptor fetch / release: the reducer holding the descriptor (gpu::reducer_holder_id); carried
  // in the RTS path field on the wire
  std::string holder;
};

struct FetchAck {
  int status = 0;          // 0 ok, <0 error (unknown MOF, I/O error, path too long)
  int64_t raw_len = 0;
  int64_t part_len = 0;
  int64_t sent = 0;        // bytes written into the client buffer by this request
  int64_t mof_offset = 0;
  std::string path;
  std::string error;
};

constexpr int kMofPathMax = 600;       // NETLEV_MOF_PATH_MAX_SIZE (NetlevComm.h:31)
// FetchRequest.buf_len of a descriptor fetch: the provider answers with the partition's device
// address in FetchAck.path (see csrc/gpu/device_ptr.h) and sends no bytes; a MOF that is not
// device-resident answers kNotDeviceResident and the reducer fetches bytes instead.
constexpr int64_t kDescriptorFetch = -1;
// FetchRequest.buf_len of a descriptor release: the holder is done with the descriptor of
// (job, map, reduce), or with every descriptor of the job when map_id is "*". The provider may then
// free the partition's HBM copy (see csrc/gpu/mof_cache.h).
constexpr int64_t kDescriptorRelease = -2;
constexpr int kNotDeviceResident = -12;
constexpr int kFetchReqMax = 800;      // NETLEV_FETCH_REQSIZE (NetlevComm.h:30)

std::string format_rts(const FetchRequest& r, uint64_t remote_addr, uint64_t req_ptr);
bool parse_rts(const std::string& s, FetchRequest* r, uint64_t* remote_addr, uint64_t* req_ptr);
std::string format_ack(const FetchAck& a);
bool parse_ack(const std::string& s, FetchAck* a);

using FetchDone = std::function<void(const FetchAck& ack)>;

// Provider side: serve one request by writing up to req.buf_len bytes of the partition
// (starting at req.fetched) into `dst`, then calling `done` (possibly from another thread).
class DataServer {
 public:
  virtual ~DataServer() = default;
  virtual void serve(const FetchRequest& req, uint8_t* dst, FetchDone done) = 0;

  // The bytes of a byte fetch by reference, for a transport that sends them itself instead of copying
  // them into a buffer first: memory (ptr) or a file range (fd, file_off: sendfile). release() runs once
  // the transport is done with them (always, whatever happened to the connection).
  struct Bytes {
    const uint8_t* ptr = nullptr;
    int fd = -1;
    int64_t file_off = 0;
    std::function<void()> release;
  };
  using RefDone = std::function<void(const FetchAck& ack, Bytes bytes)>;
  // Serve `req` by reference (ack.sent bytes in `bytes`). false: this server cannot (the transport uses
  // serve() with a buffer of its own).
  virtual bool serve_ref(const FetchRequest& req, RefDone done) {
    (void)req;
    (void)done;
    return false;
  }
};

// Client side.
class ClientTransport {
 public:
  virtual ~ClientTransport() = default;
  // Asynchronously fetch into dst (capacity req.buf_len). `done` runs on a transport thread.
  virtual void fetch(const std::string& host, const FetchRequest& req, uint8_t* dst, FetchDone done) = 0;
  virtual void close() {}
  virtual const char* name() const = 0;
};

// Server side endpoint that feeds a DataServer.
class ServerTransport {
 public:
  virtual ~ServerTransport() = default;
  virtual void start(DataServer* server) = 0;
  virtual void stop() = 0;
  virtual int port() const { return -1; }
};

// In-process registry of providers by host name (loopback backend).
void loopback_register(const std::string& host, DataServer* server);
void loopback_unregister(const std::string& host, DataServer* server);
std::unique_ptr<ClientTransport> make_loopback_client();
std::unique_ptr<ServerTransport> make_loopback_server(const std::string& host);

// TCP backend. The server listens on `port` (0 = ephemeral); clients connect to host:port with
// up to `credits` requests in flight per connection.
// bind_addr: IPv4 listen address ("" = any). Several providers on one host (one per GPU) listen on
// the same port at different addresses, as providers on different hosts do.
std::unique_ptr<ServerTransport> make_tcp_server(int port, int credits, const std::string& bind_addr = std::string());
// connections: sockets per provider host; requests go to the one with the fewest in flight (the
// credits apply per socket). One stream over loopback or a NIC queue moves ~5 GB/s; several move the
// partition bytes in parallel (the reference spreads them over RDMA QPs of one connection).
std::unique_ptr<ClientTransport> make_tcp_client(int default_port, int credits, int connections = 4);
// A process hosting both a provider and reduce tasks (the node merge service): TCP fetches that name a
// provider of this process (a local address and its port) are served in process, zero-copy.
void set_tcp_local_bypass(bool on);

// Fault injection for tests (env UDA_FAULT_FETCH=<n>: the n-th fetch fails; see uda/fault.h).
bool fault_should_fail_fetch();

}  // namespace uda
