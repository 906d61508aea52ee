// Host side of the F6 block-decompress stage: frames Hadoop block-compressed streams into per-block
// decode descriptors and runs the device decoder (csrc/gpu/decode.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "device_engine.h"
#include "kernels.h"
#include "uda/codec.h"

namespace uda {
namespace gpu {

struct BlockPlan {
  std::vector<DecodeDesc> descs;       // all blocks of all streams, dst offsets into one output buffer
  std::vector<int64_t> raw_offset;     // per stream: first raw byte (size streams + 1)
  int64_t raw_total = 0;
};

// Walk the framing of each stream (`offs[i]`..`offs[i]+lens[i]` of one host buffer, or of separate
// buffers when ptrs is given). Returns false when the framing cannot be resolved without decoding
// (an LZO block split into several chunks) or is malformed; the caller then decodes on the host.
bool plan_block_streams(Codec codec, const std::vector<const uint8_t*>& ptrs, const std::vector<int64_t>& lens,
                        BlockPlan* plan);

// Same plan for streams that live in device memory (HBM-resident compressed map outputs): the framing
// is walked on the device (launch_frame_streams) and the descriptors carry absolute source
// addresses, so decode() takes d_in = nullptr and reads every stream where it lies. false: the
// framing needs a decode (the caller falls back to the host path). Synchronizes s.
bool plan_block_streams_device(Codec codec, const std::vector<const uint8_t*>& dptrs, const std::vector<int64_t>& lens,
                               BlockPlan* plan, DeviceBuffer& scratch, DeviceBuffer& desc_scratch, hipStream_t s);

class DeviceBlockDecoder {
 public:
  // d_in: device copy of the streams back to back (stream i at sum(lens[<i])), or nullptr for a plan
  // with absolute source addresses (plan_block_streams_device); d_out: raw_total bytes.
  // Throws UdaError on a corrupt block. Synchronizes s.
  void decode(Codec codec, const BlockPlan& plan, const uint8_t* d_in, uint8_t* d_out, hipStream_t s);

 private:
  DeviceBuffer descs_, status_;
};

}  // namespace gpu
}  // namespace uda
