// TeraGen-shaped synthetic map-output generation and key-range round splitting (gfx950).
//
// Reference context: the regression harness generates input with teragen, 10^7 rows x 100 B per
// "GB" (scripts/regression/defaultsConf.sh:81); map tasks sort and spill one IFile partition per
// reducer. Here the map side's sorted per-partition runs are produced directly in HBM: each run is
// a TeraSort IFile stream (104-byte records, Text key of 10 bytes, Text value of 90 bytes) followed
// by the EOF marker, with keys stratified over the reducer's key range plus uniform jitter so that
// the runs of one reducer interleave randomly (what a range-partitioned TeraSort produces).
#include "kernels.h"

namespace uda {
namespace gpu {

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Eight printable value bytes from one random word (letters 'A'..'Z' like TeraGen's filler).
__device__ __forceinline__ uint64_t printable8(uint64_t r) {
  uint64_t w = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    uint64_t c = 'A' + ((r >> (b * 8)) & 0xFF) % 26;
    w |= c << (b * 8);
  }
  return w;
}

__global__ void __launch_bounds__(256) teragen_kernel(uint8_t* const* bases, const int64_t* nrec,
                                                      const uint64_t* key_lo,
                                                      const uint64_t* key_span,
                                                      const uint64_t* seeds,
                                                      unsigned long long* run_checksum, int unsorted) {
  const int r = blockIdx.y;
  const int64_t n = nrec[r];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long h = 0;
  if (i < n) {
    uint8_t* rec = bases[r] + i * kTeraRecordBytes;
    uint64_t st = seeds[r] ^ (0xD1B54A32D192ED03ULL * (uint64_t)(i + 1));
    const uint64_t span = key_span[r];
    const uint64_t stride = span / (uint64_t)n;
    uint64_t hi;
    if (unsorted) {  // map input: keys in generation order, sorted by launch_sort_fixed_run
      const uint64_t draw = splitmix64(st);
      hi = key_lo[r] + (span == ~0ull ? draw : draw % span);
    } else {
      const uint64_t jitter = stride ? splitmix64(st) % stride : 0;
      hi = key_lo[r] + (uint64_t)i * stride + jitter;
    }
    const uint64_t lo16 = splitmix64(st) & 0xFFFF;
    // Record layout: [0x0B keyLen=11][0x5B valLen=91][0x0A][k0..k9][0x5A][v0..v89]
    uint64_t w[13];
    // key bytes big-endian: k0..k7 = hi, k8..k9 = lo16
    uint8_t k[10];
#pragma unroll
    for (int b = 0; b < 8; ++b) k[b] = (uint8_t)(hi >> (56 - 8 * b));
    k[8] = (uint8_t)(lo16 >> 8);
    k[9] = (uint8_t)lo16;
    w[0] = 0x0Bull | (0x5Bull << 8) | (0x0Aull << 16) | ((uint64_t)k[0] << 24) |
           ((uint64_t)k[1] << 32) | ((uint64_t)k[2] << 40) | ((uint64_t)k[3] << 48) |
           ((uint64_t)k[4] << 56);
    const uint64_t v0 = printable8(splitmix64(st));
    w[1] = (uint64_t)k[5] | ((uint64_t)k[6] << 8) | ((uint64_t)k[7] << 16) |
           ((uint64_t)k[8] << 24) | ((uint64_t)k[9] << 32) | (0x5Aull << 40) |
           ((v0 & 0xFFFF) << 48);
#pragma unroll
    for (int j = 2; j < 13; ++j) w[j] = printable8(splitmix64(st));
    uint64_t* dst = reinterpret_cast<uint64_t*>(rec);
    uint64_t hh = 0x9E3779B97F4A7C15ULL ^ (uint64_t)kTeraRecordBytes;
#pragma unroll
    for (int j = 0; j < 13; ++j) {
      dst[j] = w[j];
      hh = mix64(hh ^ w[j]);
    }
    h = hh;
    if (i == n - 1) {  // IFile EOF marker VInt(-1) VInt(-1)
      rec[kTeraRecordBytes] = 0xFF;
      rec[kTeraRecordBytes + 1] = 0xFF;
    }
  }
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(run_checksum + r, h);
}

// FIXED10 key of record i of a run (hi = key bytes 0..7 BE, lo16 = key bytes 8..9).
__device__ __forceinline__ void load_fixed_key(const uint8_t* rec, uint64_t* hi, uint64_t* lo16) {
  const uint64_t w0 = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(rec));
  const uint64_t w1 = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(rec + 8));
  *hi = (w0 << 24) | (w1 >> 40);
  *lo16 = (w1 >> 24) & 0xFFFF;
}

__global__ void __launch_bounds__(256) split_fixed_kernel(uint8_t* const* bases, const int64_t* nrec,
                                                          const Elem* bounds,
                                                          const int* run_bound_set, int nruns,
                                                          int nb, int64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = nb + 2;
  if (t >= (int64_t)nruns * per) return;
  const int r = (int)(t / per);
  const int b = (int)(t % per);
  const int64_t n = nrec[r];
  if (b == 0) {
    out[t] = 0;
    return;
  }
  if (b == nb + 1) {
    out[t] = n;
    return;
  }
  const Elem bound = bounds[(int64_t)run_bound_set[r] * nb + (b - 1)];
  const uint8_t* base = bases[r];
  int64_t lo = 0, hi = n;
  while (lo < hi) {  // first record with key >= bound
    const int64_t mid = (lo + hi) >> 1;
    uint64_t kh, kl;
    load_fixed_key(base + mid * kTeraRecordBytes, &kh, &kl);
    const bool less = (kh < bound.hi) || (kh == bound.hi && kl < (bound.lo >> 48));
    if (less)
      lo = mid + 1;
    else
      hi = mid;
  }
  out[t] = lo;
}

__global__ void __launch_bounds__(256) sample_fixed_kernel(uint8_t* const* bases, const int64_t* nrec,
                                                           int nruns, int64_t every,
                                                           const int64_t* sample_off, int64_t total,
                                                           Elem* out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  int lo = 0, hi = nruns;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (sample_off[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  const int64_t i = (g - sample_off[lo]) * every + every / 2;
  if (i >= nrec[lo]) return;
  uint64_t kh, kl;
  load_fixed_key(bases[lo] + i * kTeraRecordBytes, &kh, &kl);
  out[g].hi = kh;
  out[g].lo = kl << 48;
}

// First full record's key of every block of a block-compressed FIXED10 stream, from the block's decoded
// prefix (prefix + b * slot; the record starts first_off[b] bytes in, -1: no whole key in the block).
__global__ void __launch_bounds__(256) block_first_keys_kernel(const uint8_t* prefix, int64_t slot,
                                                               const int32_t* first_off, int n, Elem* out,
                                                               int* bad) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const int f = first_off[b];
  if (f < 0) {
    out[b] = Elem{~0ull, ~0ull};
    return;
  }
  const uint8_t* r = prefix + (int64_t)b * slot + f;
  if (r[0] != 0x0B || r[1] != 0x5B || r[2] != 0x0A) {  // not the TeraSort record layout
    atomicOr(bad, 1);
    out[b] = Elem{~0ull, ~0ull};
    return;
  }
  uint64_t hi = 0;
  for (int i = 0; i < 8; ++i) hi = (hi << 8) | r[kTeraKeyOffset + i];
  const uint64_t lo16 = ((uint64_t)r[kTeraKeyOffset + 8] << 8) | r[kTeraKeyOffset + 9];
  out[b] = Elem{hi, lo16 << 48};
}

}  // namespace

void launch_block_first_keys(const uint8_t* prefix, int64_t slot, const int32_t* first_off, int n, Elem* out, int* bad,
                             hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(block_first_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, prefix, slot,
                     first_off, n, out, bad);
}

void launch_sample_fixed(uint8_t* const* bases, const int64_t* nrec, int nruns, int64_t every,
                         const int64_t* sample_off, int64_t total, Elem* out, hipStream_t s) {
  if (total <= 0) return;
  hipLaunchKernelGGL(sample_fixed_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     bases, nrec, nruns, every, sample_off, total, out);
}

void launch_teragen(uint8_t* const* bases, const int64_t* nrec, const uint64_t* key_lo,
                    const uint64_t* key_span, const uint64_t* seeds, int nruns, int64_t max_nrec,
                    unsigned long long* run_checksum, hipStream_t s, int unsorted) {
  if (nruns <= 0 || max_nrec <= 0) return;
  dim3 grid((unsigned)((max_nrec + 255) / 256), (unsigned)nruns);
  hipLaunchKernelGGL(teragen_kernel, grid, dim3(256), 0, s, bases, nrec, key_lo, key_span, seeds,
                     run_checksum, unsorted);
}

void launch_split_fixed(uint8_t* const* bases, const int64_t* nrec, const Elem* bounds,
                        const int* run_bound_set, int nruns, int nb, int64_t* out, hipStream_t s) {
  const int64_t total = (int64_t)nruns * (nb + 2);
  if (total <= 0) return;
  hipLaunchKernelGGL(split_fixed_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     bases, nrec, bounds, run_bound_set, nruns, nb, out);
}

}  // namespace gpu
}  // namespace uda
