// D2H ceiling probe, second method: compare the runtime copy path (hipMemcpyAsync, as bench.py uses)
// against a kernel that stores straight into pinned host memory over PCIe (zero-copy writes), for
// coherent and non-coherent pinned allocations and several grid sizes. Prints one JSON object.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/d2h_kernel_probe tools/d2h_kernel_probe.hip
//   /tmp/d2h_kernel_probe [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) store_to_host(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                     long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(src[i], &dst[i]);
}

static float time_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? std::atof(argv[1]) : 4.0;
  const size_t bytes = (size_t)(gib * (1ull << 30)) & ~((size_t)(1 << 20) - 1);
  const long n16 = (long)(bytes / 16);
  void* d = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 0x5a, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned flags[2] = {hipHostMallocDefault, hipHostMallocNonCoherent};
  const char* fname[2] = {"coherent", "noncoherent"};
  std::printf("{\"bytes\": %zu", bytes);
  for (int f = 0; f < 2; ++f) {
    void* h = nullptr;
    CK(hipHostMalloc(&h, bytes, flags[f]));
    std::memset(h, 0, bytes);
    const int reps = 3;
    // runtime copy path, 1 MiB pieces (the bench's delivery granularity) and one big copy
    for (int piece_mb : {1, 16, 0}) {
      const size_t piece = piece_mb ? ((size_t)piece_mb << 20) : bytes;
      CK(hipMemcpyAsync(h, d, piece, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r)
        for (size_t off = 0; off < bytes; off += piece)
          CK(hipMemcpyAsync((char*)h + off, (char*)d + off, piece, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      std::printf(", \"%s_memcpy_%s\": %.2f", fname[f], piece_mb ? (piece_mb == 1 ? "1MiB" : "16MiB") : "whole",
                  reps * bytes / (time_ms(e0, e1) * 1e-3) / 1e9);
    }
    // 512 MiB pieces at record-aligned (104 B) vs 4 KiB-aligned offsets: does alignment pick the engine?
    for (size_t shift : {(size_t)104, (size_t)4096}) {
      const size_t piece = (size_t)512 << 20;
      const int np = (int)((bytes - shift) / piece);
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r)
        for (int i = 0; i < np; ++i)
          CK(hipMemcpyAsync((char*)h + shift + i * piece, (char*)d + shift + i * piece, piece - 104,
                            hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      std::printf(", \"%s_memcpy_512MiB_off%zu\": %.2f", fname[f], shift,
                  (double)reps * np * (piece - 104) / (time_ms(e0, e1) * 1e-3) / 1e9);
    }
    for (int blocks : {256, 1024, 4096, 16384}) {
      store_to_host<<<blocks, 256, 0, s>>>((const v4u*)d, (v4u*)h, n16);
      CK(hipGetLastError());
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) store_to_host<<<blocks, 256, 0, s>>>((const v4u*)d, (v4u*)h, n16);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      std::printf(", \"%s_kernel_%dwg\": %.2f", fname[f], blocks, reps * bytes / (time_ms(e0, e1) * 1e-3) / 1e9);
    }
    // spot check the kernel's output
    const unsigned char* hb = (const unsigned char*)h;
    if (hb[0] != 0x5a || hb[bytes - 1] != 0x5a) {
      std::fprintf(stderr, "bad host data\n");
      return 1;
    }
    CK(hipHostFree(h));
  }
  std::printf("}\n");
  CK(hipFree(d));
  return 0;
}
