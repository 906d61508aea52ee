// Pinned host memory for the fetch arena, N x 256 MiB, four ways: hipHostMalloc one after another,
// hipHostMalloc from N threads, and mmap + first touch from N threads (optionally MADV_HUGEPAGE) then
// hipHostRegister. Does the pinning scale, and what does the registration alone cost once the pages
// exist? Prints one JSON line.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double mmap_register(int n, size_t bytes, bool huge, double* touch_ms) {
  std::vector<void*> p(n, nullptr);
  double t0 = now_ms();
  for (int i = 0; i < n; ++i) {
    p[i] = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p[i] == MAP_FAILED) return -1;
    if (huge) (void)madvise(p[i], bytes, MADV_HUGEPAGE);
  }
  std::vector<std::thread> ts;
  for (int i = 0; i < n; ++i) ts.emplace_back([&, i] { std::memset(p[i], 0, bytes); });
  for (auto& t : ts) t.join();
  *touch_ms = now_ms() - t0;
  t0 = now_ms();
  for (int i = 0; i < n; ++i)
    if (hipHostRegister(p[i], bytes, hipHostRegisterDefault) != hipSuccess) return -2;
  const double reg = now_ms() - t0;
  for (int i = 0; i < n; ++i) {
    (void)hipHostUnregister(p[i]);
    munmap(p[i], bytes);
  }
  return reg;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const size_t bytes = (size_t)256 << 20;
  if (hipSetDevice(0) != hipSuccess) return 1;
  (void)hipFree(nullptr);
  std::vector<void*> p(n, nullptr);
  double t0 = now_ms();
  for (int i = 0; i < n; ++i)
    if (hipHostMalloc(&p[i], bytes, hipHostMallocDefault) != hipSuccess) return 2;
  const double serial = now_ms() - t0;
  for (void* q : p) (void)hipHostFree(q);
  t0 = now_ms();
  std::vector<std::thread> ts;
  for (int i = 0; i < n; ++i)
    ts.emplace_back([&, i] { (void)hipHostMalloc(&p[i], bytes, hipHostMallocDefault); });
  for (auto& t : ts) t.join();
  const double par = now_ms() - t0;
  for (void* q : p) (void)hipHostFree(q);
  double touch4k = 0, touch2m = 0;
  const double reg4k = mmap_register(n, bytes, false, &touch4k);
  const double reg2m = mmap_register(n, bytes, true, &touch2m);
  std::printf("{\"blocks\": %d, \"mib_each\": 256, \"hipHostMalloc_serial_ms\": %.1f, \"hipHostMalloc_threads_ms\": %.1f, "
              "\"mmap_touch_threads_ms\": %.1f, \"register_ms\": %.1f, \"mmap_hugepage_touch_threads_ms\": %.1f, "
              "\"register_hugepage_ms\": %.1f}\n",
              n, serial, par, touch4k, reg4k, touch2m, reg2m);
  return 0;
}
