// Secondary-sort map outputs generated on the device (BASELINE config #5 at scale): variable-length
// Text keys sharing long common prefixes, skewed partition sizes.
//
// Key content of record i of a run: "user/" d4(f) "/s/" 'x' * pad(f) d10(seq), with f = v / 1e10,
// seq = v % 1e10 and v stratified over [0, 64e10) with random jitter (v_i strictly ascends with i,
// so every run is sorted). pad(f) = (37 f) mod 41 gives 22..62-byte keys whose first 12 bytes are
// shared by a whole family and whose first 5 by all keys: the 8-byte normalized prefix cannot order
// them, every merge comparison falls through to the full key bytes. Values: 0..120 random bytes.
// The same model as the host generator uda_amd/utils/datagen.secondary_sort (prefix families +
// numeric suffix, Pareto skew to reducer 0), sized for tens of GB.
#include "secgen.h"

#include <algorithm>
#include <stdexcept>

#include "device_engine.h"
#include "kernels.h"

namespace uda {
namespace gpu {

namespace {
constexpr uint64_t kPerFamily = 10000000000ull;  // 1e10 sequence numbers per family
constexpr uint64_t kFamilies = 64;

__device__ __forceinline__ uint64_t h64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct RecShape {
  uint64_t v;
  int pad, klen, vlen;
};

__device__ __forceinline__ RecShape shape(uint64_t seed, int64_t i, int64_t n) {
  RecShape s;
  const uint64_t space = kFamilies * kPerFamily;
  const uint64_t r = h64(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(i + 1)));
  // stratum [i*space/n, (i+1)*space/n) with jitter inside it (128-bit free: space/n fits 64 bits)
  const uint64_t step = space / (uint64_t)n;
  const uint64_t base = (uint64_t)i * step;
  s.v = base + (step > 1 ? (r >> 8) % step : 0);
  const int f = (int)(s.v / kPerFamily);
  s.pad = (37 * f) % 41;
  s.klen = 5 + 4 + 3 + s.pad + 10;
  s.vlen = (int)((r & 0xFF) % 121);
  return s;
}

__device__ __forceinline__ int64_t rec_size(const RecShape& s) { return 2 + 1 + s.klen + 1 + s.vlen; }

// bytes[r] += sizes of run r's records (runs of one map: r = partition)
__global__ void __launch_bounds__(256) secgen_bytes_kernel(const uint64_t* seeds, const int64_t* nrec, int nruns,
                                                           unsigned long long* bytes) {
  const int r = blockIdx.y;
  const int64_t n = nrec[r];
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)rec_size(shape(seeds[r], i, n));
  // wave reduce then one atomic per wave
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(&bytes[r], acc);
}

// sizes[rec_first[r] + i] = size of record i of run r
__global__ void __launch_bounds__(256) secgen_sizes_kernel(const uint64_t* seeds, const int64_t* nrec,
                                                           const int64_t* rec_first, int64_t* sizes) {
  const int r = blockIdx.y;
  const int64_t n = nrec[r];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    sizes[rec_first[r] + i] = rec_size(shape(seeds[r], i, n));
}

__device__ __forceinline__ void put_dec(uint8_t* p, uint64_t v, int digits) {
  for (int d = digits - 1; d >= 0; --d) {
    p[d] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
}

// record i of run r at base + off[rec_first[r] + i] + 2 * r (the EOF markers of the runs before it)
__global__ void __launch_bounds__(256) secgen_write_kernel(const uint64_t* seeds, const int64_t* nrec,
                                                           const int64_t* rec_first, const int64_t* off, uint8_t* base) {
  const int r = blockIdx.y;
  const int64_t n = nrec[r];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const RecShape s = shape(seeds[r], i, n);
    uint8_t* p = base + off[rec_first[r] + i] + 2 * (int64_t)r;
    p[0] = (uint8_t)(1 + s.klen);  // IFile key length (Text: VInt + content)
    p[1] = (uint8_t)(1 + s.vlen);
    p[2] = (uint8_t)s.klen;        // Text VInt
    uint8_t* k = p + 3;
    k[0] = 'u', k[1] = 's', k[2] = 'e', k[3] = 'r', k[4] = '/';
    put_dec(k + 5, s.v / kPerFamily, 4);
    k[9] = '/', k[10] = 's', k[11] = '/';
    for (int j = 0; j < s.pad; ++j) k[12 + j] = 'x';
    put_dec(k + 12 + s.pad, s.v % kPerFamily, 10);
    uint8_t* v = k + s.klen;
    v[0] = (uint8_t)s.vlen;
    uint64_t w = h64(s.v ^ seeds[r]);
    for (int j = 0; j < s.vlen; ++j) {
      if ((j & 7) == 0 && j) w = h64(w);
      v[1 + j] = (uint8_t)(w >> (8 * (j & 7)));
    }
  }
}

__global__ void secgen_eof_kernel(const int64_t* eof_at, int nruns, uint8_t* base) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  base[eof_at[r]] = 0xFF;
  base[eof_at[r] + 1] = 0xFF;
}
}  // namespace

SecGenPlan secgen_plan(int maps, int partitions, int64_t records_per_map, double skew, uint64_t seed,
                       int hot_every) {
  SecGenPlan p;
  p.maps = maps;
  p.partitions = partitions;
  p.seed = seed;
  p.nrec.assign((size_t)maps * partitions, 0);
  if (hot_every <= 0 || hot_every > partitions) hot_every = partitions;
  const int nhot = (partitions + hot_every - 1) / hot_every, ncold = partitions - nhot;
  for (int m = 0; m < maps; ++m) {
    int64_t* n = &p.nrec[(size_t)m * partitions];
    if (ncold == 0) {  // every partition hot (one partition): an even split
      for (int q = 0; q < partitions; ++q) n[q] = records_per_map / partitions + (q < records_per_map % partitions);
      continue;
    }
    const int64_t hot = (int64_t)((double)records_per_map * skew);
    const int64_t rest = records_per_map - hot;
    for (int q = 0, h = 0, c = 0; q < partitions; ++q) {
      if (q % hot_every == 0) {
        n[q] = hot / nhot + (h < hot % nhot ? 1 : 0);
        ++h;
      } else {
        n[q] = rest / ncold + (c < rest % ncold ? 1 : 0);
        ++c;
      }
    }
  }
  // per-run byte sizes on the device (records + EOF)
  const int R = maps * partitions;
  std::vector<uint64_t> seeds((size_t)R);
  for (int r = 0; r < R; ++r) seeds[(size_t)r] = seed ^ (0xC2B2AE3D27D4EB4Full * (uint64_t)(r + 1));
  DeviceBuffer d_seed((size_t)R * 8), d_n((size_t)R * 8), d_b((size_t)R * 8);
  HIP_CHECK(hipMemcpy(d_seed.as(), seeds.data(), (size_t)R * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(d_n.as(), p.nrec.data(), (size_t)R * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemset(d_b.as(), 0, (size_t)R * 8));
  for (int r0 = 0; r0 < R; r0 += 65535) {
    const int nr = std::min(65535, R - r0);
    hipLaunchKernelGGL(secgen_bytes_kernel, dim3(256, (unsigned)nr), dim3(256), 0, 0, d_seed.as<uint64_t>() + r0,
                       d_n.as<int64_t>() + r0, nr, d_b.as<unsigned long long>() + r0);
  }
  HIP_CHECK(hipGetLastError());
  std::vector<uint64_t> b((size_t)R);
  HIP_CHECK(hipMemcpy(b.data(), d_b.as(), (size_t)R * 8, hipMemcpyDeviceToHost));
  p.part_bytes.resize((size_t)R);
  p.mof_off.assign((size_t)maps + 1, 0);
  int64_t off = 0;
  for (int m = 0; m < maps; ++m) {
    p.mof_off[(size_t)m] = off;
    for (int q = 0; q < partitions; ++q) {
      p.part_bytes[(size_t)m * partitions + q] = (int64_t)b[(size_t)m * partitions + q] + 2;
      off += p.part_bytes[(size_t)m * partitions + q];
    }
    off = (off + 255) / 256 * 256;
  }
  p.mof_off[(size_t)maps] = off;
  p.seeds = seeds;
  return p;
}

void secgen_write(const SecGenPlan& p, uint8_t* store, hipStream_t s) {
  const int P = p.partitions;
  int64_t max_recs = 0;
  for (int m = 0; m < p.maps; ++m) {
    int64_t n = 0;
    for (int q = 0; q < P; ++q) n += p.nrec[(size_t)m * P + q];
    max_recs = std::max(max_recs, n);
  }
  DeviceBuffer d_seed((size_t)P * 8), d_n((size_t)P * 8), d_first((size_t)P * 8), d_eof((size_t)P * 8),
      sizes((size_t)std::max<int64_t>(max_recs, 1) * 8), offs((size_t)(max_recs + 1) * 8),
      tmp((size_t)scan_tmp_elems(std::max<int64_t>(max_recs, 1)) * 8);
  for (int m = 0; m < p.maps; ++m) {
    std::vector<int64_t> first((size_t)P + 1, 0), eof((size_t)P, 0);
    int64_t at = p.mof_off[(size_t)m];
    for (int q = 0; q < P; ++q) {
      first[(size_t)q + 1] = first[(size_t)q] + p.nrec[(size_t)m * P + q];
      at += p.part_bytes[(size_t)m * P + q];
      eof[(size_t)q] = at - 2;
    }
    HIP_CHECK(hipMemcpyAsync(d_seed.as(), p.seeds.data() + (size_t)m * P, (size_t)P * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_n.as(), p.nrec.data() + (size_t)m * P, (size_t)P * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_first.as(), first.data(), (size_t)P * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_eof.as(), eof.data(), (size_t)P * 8, hipMemcpyHostToDevice, s));
    const int64_t n = first[(size_t)P];
    for (int q0 = 0; q0 < P; q0 += 65535) {
      const int nq = std::min(65535, P - q0);
      hipLaunchKernelGGL(secgen_sizes_kernel, dim3(512, (unsigned)nq), dim3(256), 0, s, d_seed.as<uint64_t>() + q0,
                         d_n.as<int64_t>() + q0, d_first.as<int64_t>() + q0, sizes.as<int64_t>());
    }
    if (n > 0) launch_exclusive_scan(sizes.as<int64_t>(), offs.as<int64_t>(), n, tmp.as<int64_t>(), s);
    for (int q0 = 0; q0 < P; q0 += 65535) {
      const int nq = std::min(65535, P - q0);
      // base is the MOF start; record offsets already include the earlier partitions' records, the
      // kernel adds 2 bytes per earlier EOF marker (run index r = q)
      hipLaunchKernelGGL(secgen_write_kernel, dim3(512, (unsigned)nq), dim3(256), 0, s, d_seed.as<uint64_t>() + q0,
                         d_n.as<int64_t>() + q0, d_first.as<int64_t>() + q0, offs.as<int64_t>(),
                         store + p.mof_off[(size_t)m] + 2 * (int64_t)q0);
    }
    hipLaunchKernelGGL(secgen_eof_kernel, dim3((unsigned)((P + 63) / 64)), dim3(64), 0, s, d_eof.as<int64_t>(), P, store);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));  // the scan scratch is reused by the next map
  }
}

}  // namespace gpu
}  // namespace uda
