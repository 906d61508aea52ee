// Kernel launches in a process on the system HIP runtime (no torch): one kernel of this executable,
// then kernels inside libuda.so. Prints the status of each; tells a runtime that cannot launch the
// library's kernels from a problem of one call site.
#include <hip/hip_runtime.h>

#include <cstdio>

namespace uda {
namespace gpu {
void launch_max_i32(const int32_t* v, int64_t n, unsigned int* out, hipStream_t s);
}
}  // namespace uda

__global__ void probe_kernel(int* p) { p[threadIdx.x] = threadIdx.x; }

int main() {
  int* d = nullptr;
  printf("hipMalloc: %s\n", hipGetErrorString(hipMalloc(&d, 4096)));
  hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(64), 0, 0, d);
  printf("own kernel launch: %s\n", hipGetErrorString(hipGetLastError()));
  printf("sync: %s\n", hipGetErrorString(hipDeviceSynchronize()));
  uda::gpu::launch_max_i32(reinterpret_cast<int32_t*>(d), 16, reinterpret_cast<unsigned int*>(d + 512), nullptr);
  printf("libuda kernel launch: %s\n", hipGetErrorString(hipGetLastError()));
  printf("sync: %s\n", hipGetErrorString(hipDeviceSynchronize()));
  int rt = 0, drv = 0;
  hipRuntimeGetVersion(&rt);
  hipDriverGetVersion(&drv);
  printf("runtime %d driver %d\n", rt, drv);
  return 0;
}
