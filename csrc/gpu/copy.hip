// Batched device copies: pack the per-destination slices of a shuffle round into one contiguous
// send region (and the self partition straight into the receive slot) with one launch.
#include "kernels.h"

namespace uda {
namespace gpu {

namespace {
constexpr int kCopyThreads = 256;

__global__ void __launch_bounds__(kCopyThreads) batched_copy_kernel(const CopyDesc* descs) {
  const CopyDesc d = descs[blockIdx.y];
  const int64_t n = d.bytes;
  if (n <= 0) return;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const uintptr_t a = (uintptr_t)d.src | (uintptr_t)d.dst;
  if ((a & 15) == 0) {
    const int64_t n16 = n >> 4;
    const uint4* s = reinterpret_cast<const uint4*>(d.src);
    uint4* t = reinterpret_cast<uint4*>(d.dst);
    for (int64_t i = tid; i < n16; i += stride) t[i] = s[i];
    for (int64_t i = (n16 << 4) + tid; i < n; i += stride) d.dst[i] = d.src[i];
  } else if ((a & 7) == 0) {
    const int64_t n8 = n >> 3;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(d.src);
    uint64_t* t = reinterpret_cast<uint64_t*>(d.dst);
    for (int64_t i = tid; i < n8; i += stride) t[i] = s[i];
    for (int64_t i = (n8 << 3) + tid; i < n; i += stride) d.dst[i] = d.src[i];
  } else {
    for (int64_t i = tid; i < n; i += stride) d.dst[i] = d.src[i];
  }
}
}  // namespace

void launch_batched_copy(const CopyDesc* descs, int n, int64_t max_bytes, hipStream_t s, int max_blocks) {
  if (n <= 0 || max_bytes <= 0) return;
  // enough workgroups per descriptor to keep ~16 KiB per workgroup, capped for huge slices
  int64_t blocks = (max_bytes + (16 << 10) - 1) / (16 << 10);
  if (blocks > max_blocks) blocks = max_blocks;
  hipLaunchKernelGGL(batched_copy_kernel, dim3((unsigned)blocks, (unsigned)n), dim3(kCopyThreads), 0, s, descs);
}

}  // namespace gpu
}  // namespace uda
