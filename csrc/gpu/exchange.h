// Device all-to-all-v exchange used by the shuffle rounds.
//
// Reference analogue: the M x R point-to-point RDMA WRITEs of MOF chunks into reducer buffers
// (src/DataNet/RDMAServer.cc:537-631 rdma_write_mof_send_ack, src/DataNet/RDMAClient.cc:559-600
// start_fetch_req). On MI355X one round of the shuffle is an all-to-all-v over xGMI: every rank
// sends, per destination, the slices of its map outputs that fall in the round's key cells, and
// receives its own cells from every peer.
//
// Contract of exchange() (the NCCL point-to-point rules, enforced by every backend):
//   * send[p] / recv[p] are the ordered non-empty slices to / from peer p; the self entries are empty.
//   * The k-th slice this rank sends to p pairs with the k-th slice p receives from this rank: the
//     number of slices and every size must agree (a mismatch is an error, never a partial transfer).
//   * Slices are device memory (hipMalloc); host-pinned sources are refused.
//   * Send slices may be written by work enqueued on `s` before the call: every backend orders its
//     reads after it (RCCL by stream order; pull backends by an event the receivers' streams wait for,
//     or a host wait before the sender publishes its slice list).
//   * Receive slices must not be touched before the work enqueued on `s` has passed the exchange.
//   * Send slices must stay unchanged until wait_sent(seq) of that exchange returned (stream order on
//     `s` is enough for RCCL; pull-based backends read the sender's memory from the peers' streams).
// Exchanges are numbered 0, 1, 2, ... per Exchange object (seq).
//
// Implementations:
//   RcclExchange   - one process per GPU, RCCL communicator bootstrapped from an ncclUniqueId.
//                    Default (zero-copy): every slice is its own ncclSend straight from its source
//                    into its receive slot, all of a round's sends and receives inside one
//                    ncclGroupStart/End, peers in rotating order. UDA_RCCL_PACK=1 packs each peer's
//                    slices on the comm stream into one staging region and sends one message per peer.
//   IpcExchange    - one process per GPU (or several processes sharing one GPU): a node-local
//                    shared-memory control plane (uda/shm_group.h) plus pull copies straight from
//                    the peers' HBM, mapped once per allocation over hipIpc (xGMI reads between
//                    GPUs). Needs no RCCL kernels or CUs beyond the copies, and runs with N ranks on
//                    one GPU, which RCCL refuses - so the multi-process path is exercised on a
//                    one-GPU machine.
//   LocalExchange  - W ranks as threads of one process sharing a device (tests / rehearsal): each
//                    receiver pulls its slices from the senders' memory on its own stream, with the
//                    same pairing / device-memory checks as the multi-process backends.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

typedef struct ncclComm* ncclComm_t;

namespace uda {
namespace gpu {

struct Span {
  const uint8_t* ptr;
  int64_t bytes;
};

class Exchange {
 public:
  virtual ~Exchange() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // Ranks the underlying communicator reports (ncclCommCount for RCCL).
  virtual int comm_ranks() const { return world(); }
  // Blocking exchange of `n` int64 per peer: recv[p*n..] <- peer p's send[me*n..].
  virtual void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t s) = 0;
  // Size internal staging for rounds sending at most `bytes` to all peers together.
  virtual void reserve(int64_t bytes) { (void)bytes; }
  // Enqueue one all-to-all-v round on stream s (see the contract above).
  virtual void exchange(const std::vector<std::vector<Span>>& send, const std::vector<std::vector<Span>>& recv,
                        hipStream_t s) = 0;
  virtual std::string name() const = 0;
  // Host wait until every peer has finished reading what this rank sent in exchange `seq` (after
  // which those send slices may be overwritten). Stream-ordered backends return at once.
  virtual void wait_sent(int64_t seq) { (void)seq; }
  // Collective end of a step, called after this rank's streams drained: when it returns no peer
  // reads this rank's memory any more (buffers may be freed or rewritten).
  virtual void quiesce() {}
  // Host wait for everything enqueued on `s`, failing instead of hanging when a peer is lost
  // (RCCL: asynchronous communicator errors and a timeout, UDA_RCCL_TIMEOUT_S, default 900 s).
  virtual void wait(hipStream_t s);
  // Throw if the communicator reported an asynchronous error (cheap, non-blocking).
  virtual void check() {}
};

std::unique_ptr<Exchange> make_rccl_exchange(int rank, int world, const std::string& unique_id);
// All ranks of group `group` must call this with the same world; ranks are threads.
std::unique_ptr<Exchange> make_local_exchange(const std::string& group, int rank, int world);
// All ranks (processes on one node) call this with the same `name` (agreed out of band, e.g. by a
// broadcast from rank 0); collective. `device` is this rank's HIP device.
std::unique_ptr<Exchange> make_ipc_exchange(const std::string& name, int rank, int world, int device);

// Test probe: `rounds` exchanges of synthetic slices (send_sizes[p] / recv_sizes[p]: slice sizes to /
// from peer p), every received byte checked. Returns "" or the error (pairing, memory-kind, data).
// host_source: the send slices live in pinned host memory (must be refused).
// export_bytes: the send slices are spread over one device allocation of this size (a store-sized
// export: the peers map it and read beyond 4 GiB of it).
std::string exchange_probe(Exchange& ex, int device, const std::vector<std::vector<int64_t>>& send_sizes,
                           const std::vector<std::vector<int64_t>>& recv_sizes, bool host_source, int rounds,
                           int64_t export_bytes = 0);

}  // namespace gpu
}  // namespace uda
