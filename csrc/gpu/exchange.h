// Device all-to-all-v exchange used by the shuffle rounds.
//
// Reference analogue: the M x R point-to-point RDMA WRITEs of MOF chunks into reducer buffers
// (src/DataNet/RDMAServer.cc:537-631 rdma_write_mof_send_ack, src/DataNet/RDMAClient.cc:559-600
// start_fetch_req). On MI355X one round of the shuffle is an all-to-all-v over xGMI: every rank
// sends, per destination, the slices of its map outputs that fall in the round's key cells, and
// receives its own cells from every peer.
//
// Contract of exchange(): send[p] / recv[p] are the ordered non-empty slices to / from peer p
// (p != me; the self entry must be empty). The k-th slice this rank sends to p pairs with the
// k-th slice p receives from this rank; sizes must agree. Slices stay valid and unchanged until
// the enqueued work on `s` has passed this exchange.
//
// Implementations:
//   RcclExchange   - one process per GPU, RCCL communicator bootstrapped from an ncclUniqueId.
//                    Default (zero-copy): every slice is its own ncclSend straight from the map
//                    output in the store into its receive slot, all of a round's sends and
//                    receives inside one ncclGroupStart/End, peers in rotating order. A TeraSort
//                    slice is tens of MB (130 GB / (16 rounds x 8 peers x 32 maps) = 32 MB), so
//                    per-operation overhead is noise, and no CU time or HBM bandwidth goes to a pack.
//                    UDA_RCCL_PACK=1 packs each peer's slices on the comm stream into one staging
//                    region and sends one message per peer (for jobs with many tiny slices); the
//                    receiver's slices from a peer must then be contiguous.
//   LocalExchange  - W ranks as threads of one process sharing a device (tests / single-GPU
//                    rehearsal of the multi-rank schedule): each receiver pulls its slices from
//                    the senders' memory with copies on its own stream. Requires the send slices
//                    to be immutable for the whole step (true for store-resident map outputs).
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
  virtual const char* name() const = 0;
  // Host wait for everything enqueued on `s`, failing instead of hanging when a peer is lost
  // (RCCL: asynchronous communicator errors and a timeout, UDA_RCCL_TIMEOUT_S, default 900 s).
  virtual void wait(hipStream_t s);
  // Throw if the communicator reported an asynchronous error (cheap, non-blocking).
  virtual void check() {}
};

std::unique_ptr<Exchange> make_rccl_exchange(int rank, int world, const std::string& unique_id);
// All ranks of group `group` must call this with the same world; ranks are threads.
std::unique_ptr<Exchange> make_local_exchange(const std::string& group, int rank, int world);

}  // namespace gpu
}  // namespace uda
