// Where a fresh process's first GPU milliseconds go (the cold reduce task: Hadoop starts every reduce
// task in its own JVM). Phases, each timed on its own, in the order a reduce task meets them:
//   hsa      hsa_init (ROCr: KFD open, topology, agents)
//   hip      hipGetDeviceCount (the HIP runtime over ROCr)
//   ctx      hipSetDevice + hipFree(nullptr) (the device context, its blit queues)
//   malloc   hipMalloc of 4 KiB
//   launch   first launch of a libuda.so kernel + sync (the library's code object)
//   stream   hipStreamCreate
//   pin      hipHostRegister of 64 MiB of touched anonymous memory
// One JSON line on stdout. tools/probes/hip_init_probe.py starts N of these at once.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace uda {
namespace gpu {
void launch_max_i32(const int32_t* v, int64_t n, unsigned int* out, hipStream_t s);
}
}  // namespace uda

namespace {
double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_BOOTTIME, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
}  // namespace

int main() {
  const double t0 = now_ms();
  double t[8];
  int i = 0;
  const hsa_status_t hs = hsa_init();
  t[i++] = now_ms();
  int n = 0;
  const hipError_t e1 = hipGetDeviceCount(&n);
  t[i++] = now_ms();
  const hipError_t e2 = hipSetDevice(0);
  (void)hipFree(nullptr);
  t[i++] = now_ms();
  int* d = nullptr;
  const hipError_t e3 = hipMalloc(&d, 4096);
  t[i++] = now_ms();
  uda::gpu::launch_max_i32(reinterpret_cast<int32_t*>(d), 16, reinterpret_cast<unsigned int*>(d + 512), nullptr);
  const hipError_t e4 = hipDeviceSynchronize();
  t[i++] = now_ms();
  hipStream_t s = nullptr;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  t[i++] = now_ms();
  const size_t pin = 64u << 20;
  void* h = mmap(nullptr, pin, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  std::memset(h, 1, pin);
  const hipError_t e5 = hipHostRegister(h, pin, hipHostRegisterDefault);
  t[i++] = now_ms();
  const char* names[] = {"hsa", "hip", "ctx", "malloc", "launch", "stream", "pin"};
  std::printf("{\"pid\":%d,\"t0_boot_ms\":%.1f,\"devices\":%d,\"ok\":%s", (int)getpid(), t0, n,
              (hs == HSA_STATUS_SUCCESS && e1 == hipSuccess && e2 == hipSuccess && e3 == hipSuccess && e4 == hipSuccess &&
               e5 == hipSuccess)
                  ? "true"
                  : "false");
  double prev = t0;
  for (int k = 0; k < i; ++k) {
    std::printf(",\"%s_ms\":%.1f", names[k], t[k] - prev);
    prev = t[k];
  }
  std::printf(",\"total_ms\":%.1f}\n", prev - t0);
  (void)hipHostUnregister(h);
  munmap(h, pin);
  (void)hipStreamDestroy(s);
  (void)hipFree(d);
  hsa_shut_down();
  return 0;
}
