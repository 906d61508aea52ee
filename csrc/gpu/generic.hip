// GENERIC record path on gfx950: any Hadoop key class, variable-length IFile records.
//
// F1 (record index) replaces BaseSegment::nextKVInternal (src/Merger/StreamRW.cc:334-404): IFile
// framing is sequential inside a run (a record's position depends on every previous VInt), so one
// lane walks one run and all runs are walked concurrently; a count pass sizes the offset arrays.
// F2 (key normalization) replaces the comparator calls of CompareFunc.cc:70-91: one lane per record
// skips the VInt / 4-byte length prefix of the key class and packs the first 8 content bytes
// big-endian, so the merge compares integers and falls back to the raw bytes only on prefix ties
// between long keys (GenericCmp in merge.hip).
// F4 (serialize) replaces write_kv_to_stream (StreamRW.cc:151-225): an exclusive scan of record sizes
// in merged order gives every record its output offset; a wave copies 64 records at a time with
// all lanes on each record (byte-granular, records are not aligned).
#include "kernels.h"
#include "uda/compare.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {

// Walk one run; returns record count and writes record bytes (offset of the EOF marker or end).
__device__ int64_t walk_run(const uint8_t* p, int64_t n, int64_t* offsets, int64_t* rec_bytes, int* status) {
  int64_t pos = 0, cnt = 0;
  *status = 0;
  while (pos < n) {
    int64_t kl = 0, vl = 0;
    const int a = vint_decode(p + pos, (size_t)(n - pos), &kl);
    if (a == 0) {
      *status = 1;
      break;
    }
    const int b = vint_decode(p + pos + a, (size_t)(n - pos - a), &vl);
    if (b == 0) {
      *status = 1;
      break;
    }
    if (kl == -1 && vl == -1) break;  // EOF marker
    if (kl < 0 || vl < 0 || pos + a + b + kl + vl > n) {
      *status = 2;
      break;
    }
    if (offsets) offsets[cnt] = pos;
    pos += a + b + kl + vl;
    ++cnt;
  }
  if (offsets) offsets[cnt] = pos;
  *rec_bytes = pos;
  return cnt;
}

__global__ void count_records_kernel(uint8_t* const* bases, const int64_t* nbytes, int nruns, int64_t* counts,
                                     int64_t* rec_bytes, int* status) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  int st = 0;
  counts[r] = walk_run(bases[r], nbytes[r], nullptr, rec_bytes + r, &st);
  status[r] = st;
}

__global__ void index_records_kernel(uint8_t* const* bases, const int64_t* nbytes, int nruns,
                                     int64_t* const* offsets) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nruns) return;
  int st = 0;
  int64_t rb = 0;
  walk_run(bases[r], nbytes[r], offsets[r], &rb, &st);
}

__device__ __forceinline__ int find_run(const int64_t* elem_off, int nruns, int64_t g) {
  int lo = 0, hi = nruns;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (elem_off[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256) normalize_kernel(GenericKeyCtx ctx, const int64_t* elem_off, int nruns,
                                                        int64_t total, Elem* out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const int r = find_run(elem_off, nruns, g);
  const int64_t pos = g - elem_off[r];
  const uint8_t* rec = ctx.bases[r] + ctx.offsets[r][pos];
  int64_t kl = 0, vl = 0;
  const int a = vint_decode(rec, 9, &kl);
  const int b = vint_decode(rec + a, 9, &vl);
  const uint8_t* key = rec + a + b;
  const int o = key_content_offset((KeyKind)ctx.kind, key, (int)kl);
  const int cl = (int)kl - o;
  Elem e;
  e.hi = load_be_prefix(key + o, cl);
  const uint64_t capped = cl > 0xFFFF ? 0xFFFF : (uint64_t)cl;
  e.lo = (capped << 48) | ((uint64_t)r << 32) | (uint64_t)pos;
  out[g] = e;
}

__global__ void __launch_bounds__(256) record_sizes_kernel(GenericKeyCtx ctx, const Elem* elems, int64_t n,
                                                           int64_t* sizes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Elem e = elems[i];
  const int r = (int)((e.lo >> 32) & 0xFFFF);
  const uint64_t pos = e.lo & 0xFFFFFFFFull;
  sizes[i] = ctx.offsets[r][pos + 1] - ctx.offsets[r][pos];
}

// ---- exclusive scan: per-block reduce, scan of block sums (one block), add-back
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ int64_t block_exclusive_scan(int64_t v, int64_t* lds, int64_t* total) {
  // wave scan then cross-wave scan through LDS
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) {
      const int64_t t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kScanThreads / 64] = run;
  }
  __syncthreads();
  const int64_t excl = x - v + lds[wid];
  *total = lds[kScanThreads / 64];
  __syncthreads();
  return excl;
}

__global__ void __launch_bounds__(kScanThreads) scan_reduce_kernel(const int64_t* in, int64_t n, int64_t* partials) {
  __shared__ int64_t lds[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < n) s += in[base + k];
  int64_t total;
  block_exclusive_scan(s, lds, &total);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kScanThreads) scan_partials_kernel(int64_t* partials, int64_t nparts) {
  __shared__ int64_t lds[kScanThreads / 64 + 1];
  int64_t carry = 0;
  for (int64_t base = 0; base < nparts; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nparts ? partials[i] : 0;
    int64_t total;
    const int64_t e = block_exclusive_scan(v, lds, &total);
    if (i < nparts) partials[i] = carry + e;
    carry += total;
  }
  if (threadIdx.x == 0) partials[nparts] = carry;
}

__global__ void __launch_bounds__(kScanThreads) scan_apply_kernel(const int64_t* in, int64_t n, const int64_t* partials,
                                                                  int64_t* out) {
  __shared__ int64_t lds[kScanThreads / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (base + k < n) ? in[base + k] : 0;
    s += v[k];
  }
  int64_t total;
  int64_t run = block_exclusive_scan(s, lds, &total) + partials[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = partials[gridDim.x];
}

// ---- variable-length gather: one wave per 64 records, all lanes on each record
__global__ void __launch_bounds__(256) gather_var_kernel(GenericKeyCtx ctx, const Elem* elems, int64_t n,
                                                         const int64_t* out_off, uint8_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t rec0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
  if (rec0 >= n) return;
  const int valid = (n - rec0) < 64 ? (int)(n - rec0) : 64;
  unsigned long long src = 0;
  long long len = 0, dst = 0;
  if (lane < valid) {
    const Elem e = elems[rec0 + lane];
    const int r = (int)((e.lo >> 32) & 0xFFFF);
    const uint64_t pos = e.lo & 0xFFFFFFFFull;
    const int64_t o = ctx.offsets[r][pos];
    src = (unsigned long long)(ctx.bases[r] + o);
    len = ctx.offsets[r][pos + 1] - o;
    dst = out_off[rec0 + lane];
  }
  for (int r = 0; r < valid; ++r) {
    const uint8_t* s = reinterpret_cast<const uint8_t*>(__shfl(src, r, 64));
    const long long l = __shfl(len, r, 64);
    uint8_t* d = out + __shfl(dst, r, 64);
    for (long long i = lane; i < l; i += 64) d[i] = s[i];
  }
}

__global__ void __launch_bounds__(256) buffer_cuts_kernel(const int64_t* out_off, int64_t n, int64_t chunk,
                                                          int64_t nbuf, int64_t* cuts) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > nbuf) return;
  const int64_t target = j * chunk;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (out_off[mid] < target)
      lo = mid + 1;
    else
      hi = mid;
  }
  cuts[j] = (j == nbuf || lo >= n) ? out_off[n] : out_off[lo];  // byte offset of the cut
}

__global__ void __launch_bounds__(256) max_kernel(const int64_t* v, int64_t n, unsigned long long* out) {
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, (unsigned long long)v[i]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

}  // namespace

void launch_max_i64(const int64_t* v, int64_t n, unsigned long long* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(max_kernel, dim3((unsigned)blocks), dim3(256), 0, s, v, n, out);
}

void launch_count_records(uint8_t* const* bases, const int64_t* nbytes, int nruns, int64_t* counts,
                          int64_t* rec_bytes, int* status, hipStream_t s) {
  if (nruns <= 0) return;
  hipLaunchKernelGGL(count_records_kernel, dim3((unsigned)((nruns + 63) / 64)), dim3(64), 0, s, bases, nbytes,
                     nruns, counts, rec_bytes, status);
}

void launch_index_records(uint8_t* const* bases, const int64_t* nbytes, int nruns, int64_t* const* offsets,
                          hipStream_t s) {
  if (nruns <= 0) return;
  hipLaunchKernelGGL(index_records_kernel, dim3((unsigned)((nruns + 63) / 64)), dim3(64), 0, s, bases, nbytes,
                     nruns, offsets);
}

void launch_normalize_generic(GenericKeyCtx ctx, const int64_t* elem_off, int nruns, int64_t total, Elem* out,
                              hipStream_t s) {
  if (total <= 0) return;
  hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, ctx, elem_off,
                     nruns, total, out);
}

void launch_record_sizes(GenericKeyCtx ctx, const Elem* elems, int64_t n, int64_t* sizes, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(record_sizes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ctx, elems, n,
                     sizes);
}

int64_t scan_tmp_elems(int64_t n) { return (n + kScanTile - 1) / kScanTile + 2; }

void launch_exclusive_scan(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s) {
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int64_t), s);
    return;
  }
  const int64_t blocks = (n + kScanTile - 1) / kScanTile;
  hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)blocks), dim3(kScanThreads), 0, s, in, n, tmp);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kScanThreads), 0, s, tmp, blocks);
  hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)blocks), dim3(kScanThreads), 0, s, in, n, tmp, out);
}

void launch_gather_var(GenericKeyCtx ctx, const Elem* elems, int64_t n, const int64_t* out_off, uint8_t* out,
                       hipStream_t s) {
  if (n <= 0) return;
  const int64_t waves = (n + 63) / 64;
  hipLaunchKernelGGL(gather_var_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, ctx, elems, n,
                     out_off, out);
}

void launch_buffer_cuts(const int64_t* out_off, int64_t n, int64_t chunk, int64_t nbuf, int64_t* cuts,
                        hipStream_t s) {
  hipLaunchKernelGGL(buffer_cuts_kernel, dim3((unsigned)((nbuf + 1 + 255) / 256)), dim3(256), 0, s, out_off, n,
                     chunk, nbuf, cuts);
}

}  // namespace gpu
}  // namespace uda
