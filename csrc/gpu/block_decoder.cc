// F6 host planner: see block_decoder.h. The framing walk touches only the 4-byte headers (and the
// Snappy length varint of each chunk), so it costs O(blocks), not O(bytes).
#include "block_decoder.h"

#include <cstring>
#include <string>

#include "uda/error.h"
#include "uda/trace.h"

namespace uda {
namespace gpu {

namespace {
uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
}  // namespace

bool plan_block_streams(Codec codec, const std::vector<const uint8_t*>& ptrs, const std::vector<int64_t>& lens,
                        BlockPlan* plan) {
  plan->descs.clear();
  plan->raw_offset.assign(1, 0);
  int64_t in_base = 0, raw = 0;
  for (size_t s = 0; s < lens.size(); ++s) {
    const uint8_t* p = ptrs[s];
    const int64_t n = lens[s];
    int64_t i = 0;
    while (i < n) {
      if (i + 4 > n) return false;
      const int64_t block_raw = be32(p + i);
      i += 4;
      if (block_raw == 0) continue;  // empty block: no chunks follow
      DecodeDesc d{in_base + i, 0, raw, block_raw};
      int64_t left = block_raw;
      while (left > 0) {
        if (i + 4 > n) return false;
        const int64_t clen = be32(p + i);
        if (i + 4 + clen > n) return false;
        int64_t produced = left;  // LZO: a single chunk must produce the whole block
        if (codec == Codec::kSnappy) {
          size_t ulen = 0;
          if (!snappy_uncompressed_length(p + i + 4, (size_t)clen, &ulen)) return false;
          produced = (int64_t)ulen;
          if (produced > left || (produced == 0 && clen > 1)) return false;
        }
        i += 4 + clen;
        if (produced == 0) return false;  // would not make progress
        left -= produced;
      }
      d.src_end = in_base + i;
      plan->descs.push_back(d);
      raw += block_raw;
    }
    in_base += n;
    plan->raw_offset.push_back(raw);
  }
  plan->raw_total = raw;
  return true;
}

bool plan_block_streams_device(Codec codec, const std::vector<const uint8_t*>& dptrs, const std::vector<int64_t>& lens,
                               BlockPlan* plan, DeviceBuffer& scratch, DeviceBuffer& desc_scratch, hipStream_t s) {
  const int n = (int)dptrs.size();
  plan->descs.clear();
  plan->raw_offset.assign(1, 0);
  plan->raw_total = 0;
  if (n == 0) return true;
  // scratch: ptrs | lens | desc_first | raw_first | nblocks | raw (8 B each per stream) | status (4 B)
  const size_t tb = (size_t)n * 52 + 64;
  if (scratch.size() < tb) scratch.alloc(tb + tb / 2);
  auto* d_ptrs = scratch.as<const uint8_t*>();
  auto* d_lens = reinterpret_cast<int64_t*>(d_ptrs + n);
  int64_t* d_dfirst = d_lens + n;
  int64_t* d_rfirst = d_dfirst + n;
  int64_t* d_nb = d_rfirst + n;
  int64_t* d_raw = d_nb + n;
  int* d_status = reinterpret_cast<int*>(d_raw + n);
  HIP_CHECK(hipMemcpyAsync(d_ptrs, dptrs.data(), 8 * (size_t)n, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_lens, lens.data(), 8 * (size_t)n, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(d_status, 0, 4 * (size_t)n, s));
  launch_frame_streams(d_ptrs, d_lens, n, (int)codec, nullptr, nullptr, d_nb, d_raw, nullptr, d_status, s);
  std::vector<int64_t> nb((size_t)n), raw((size_t)n);
  std::vector<int> st((size_t)n);
  HIP_CHECK(hipMemcpyAsync(nb.data(), d_nb, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(raw.data(), d_raw, 8 * (size_t)n, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(st.data(), d_status, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  for (int i = 0; i < n; ++i)
    if (st[(size_t)i]) return false;
  std::vector<int64_t> dfirst((size_t)n), rfirst((size_t)n);
  int64_t nd = 0, rt = 0;
  for (int i = 0; i < n; ++i) {
    dfirst[(size_t)i] = nd;
    rfirst[(size_t)i] = rt;
    nd += nb[(size_t)i];
    rt += raw[(size_t)i];
    plan->raw_offset.push_back(rt);
  }
  plan->raw_total = rt;
  plan->descs.resize((size_t)nd);
  if (nd == 0) return true;
  // the caller's buffer, kept across tasks: a per-call DeviceBuffer cost a device-synchronizing hipFree
  if (desc_scratch.size() < (size_t)nd * sizeof(DecodeDesc)) desc_scratch.alloc((size_t)nd * sizeof(DecodeDesc) * 3 / 2);
  DeviceBuffer& d_descs = desc_scratch;
  HIP_CHECK(hipMemcpyAsync(d_dfirst, dfirst.data(), 8 * (size_t)n, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(d_rfirst, rfirst.data(), 8 * (size_t)n, hipMemcpyHostToDevice, s));
  launch_frame_streams(d_ptrs, d_lens, n, (int)codec, d_dfirst, d_rfirst, d_nb, d_raw, d_descs.as<DecodeDesc>(),
                       d_status, s);
  HIP_CHECK(hipMemcpyAsync(plan->descs.data(), d_descs.as(), (size_t)nd * sizeof(DecodeDesc), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return true;
}

void DeviceBlockDecoder::decode(Codec codec, const BlockPlan& plan, const uint8_t* d_in, uint8_t* d_out,
                                hipStream_t s) {
  const int n = (int)plan.descs.size();
  if (n == 0) return;
  trace::Range tr("uda.block_decode");
  const size_t bytes = (size_t)n * sizeof(DecodeDesc);
  if (descs_.size() < bytes) descs_.alloc(bytes);
  if (status_.size() < sizeof(int)) status_.alloc(sizeof(int));
  HIP_CHECK(hipMemcpyAsync(descs_.as(), plan.descs.data(), bytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(status_.as(), 0, sizeof(int), s));
  launch_block_decode((int)codec, d_in, d_out, descs_.as<DecodeDesc>(), n, status_.as<int>(), s);
  int st = 0;
  HIP_CHECK(hipMemcpyAsync(&st, status_.as(), sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (st) throw UdaError(std::string("corrupt ") + codec_name(codec) + " block (device decode)");
}

}  // namespace gpu
}  // namespace uda
