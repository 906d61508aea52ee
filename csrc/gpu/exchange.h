// Device all-to-all-v exchange used by the shuffle rounds.
//
// Reference analogue: the M x R point-to-point RDMA WRITEs. On MI355X one round
// of the shuffle is an all-to-all-v over xGMI: every rank packs, per destination, the slices of its
// map outputs that fall in the round's key range into one contiguous region, then each pair of
// ranks exchanges one message per direction (ncclSend/ncclRecv grouped: the pattern RCCL's
// all-to-all uses, so all 7 xGMI links of a GPU are driven at once).
//
// Implementations:
//   RcclExchange   - one process per GPU, RCCL communicator bootstrapped from an ncclUniqueId.
//   LocalExchange  - W ranks as threads of one process sharing a device (tests / single-GPU
//                    rehearsal of the multi-rank schedule): copies are device memcpys, and the
//                    completion semantics of a send (sender may reuse its buffer only once every
//                    receiver has copied) are reproduced with cross-stream events.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

typedef struct ncclComm* ncclComm_t;

namespace uda {
namespace gpu {

class Exchange {
 public:
  virtual ~Exchange() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // Blocking exchange of `n` int64 per peer: recv[p*n..] <- peer p's send[me*n..].
  virtual void alltoall_i64(const int64_t* send, int64_t* recv, size_t n, hipStream_t s) = 0;
  // Enqueue an all-to-all-v on stream s. Byte counts/displacements per peer; self entries must be 0.
  virtual void alltoallv(const uint8_t* send, const int64_t* send_bytes, const int64_t* send_displ,
                         uint8_t* recv, const int64_t* recv_bytes, const int64_t* recv_displ,
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
