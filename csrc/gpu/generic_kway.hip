// Single-pass K-way merge for any key class (generic IFile records): F3 of the generic merge for
// up to kGkMaxRuns runs, replacing the log2(K) pairwise passes of merge_pass_generic_lds_kernel.
//
// Reference hot loop replaced: the segment heap of the online merge (MergeQueue::next /
// PriorityQueue::downHeap, src/Merger/MergeQueue.h:238-269, 299-321) with the key comparators of
// src/Merger/CompareFunc.cc:70-91.
//
// Design (gfx950), following kway.hip for TeraSort keys:
//  * Cells by sampling, in the generic total order (content bytes, length, ordinal; no two elements
//    are equal, so duplicate-heavy keys do not inflate cells): every s-th element of every run is
//    sampled, the samples are merged by the pairwise generic passes (small), every (ns/C)-th
//    becomes a splitter. A histogram of the merged samples by run gives each splitter's rank among
//    every run's samples, so each run is split at each splitter by a search over one sample
//    interval (~log2 s probes). With s = (cap - T) / (K + 2) a cell holds at most cap elements.
//  * One workgroup per cell (256 threads, cap 1024): the cell's elements are loaded into LDS, the
//    longest common prefix P of the cell's keys is found from its slice end points (every key of
//    a cell lies between two splitters, so the keys share a long prefix when the data has one), and
//    the 24 key bytes after P are staged in LDS next to each element. The K slices are then merged
//    pairwise inside LDS (log2 K levels, merge path per thread) on 16-bit element indices, so the
//    staged keys never move; ties past P + 24 bytes go to the key bytes in HBM. The merged elements
//    are written once; F4 (sizes, scan, gather) runs on them as before.
//  * A cell above cap (not possible with the sampling bound; kept as a guard) raises a flag and the
//    host redoes the merge with the pairwise passes.
#include "generic_cmp.h"
#include "kernels.h"

namespace uda {
namespace gpu {

namespace {
constexpr int kGkThreads = 256;
constexpr int kGkItems = 4;
constexpr int kGkCap = kGkThreads * kGkItems;  // 1024 elements per cell

__device__ __forceinline__ bool generic_lt(const GenericKeyCtx& ctx, const Elem& a, const Elem& b) {
  return !generic_le(ctx, b, a);
}

__device__ __forceinline__ int find_slot(const int64_t* off, int n, int64_t g) {  // off[lo] <= g < off[lo + 1]
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// samples[soff[r] + j] = cur[eoff[r] + j * step + step / 2]
__global__ void __launch_bounds__(256) gk_sample_kernel(const Elem* cur, const int64_t* eoff, const int64_t* soff, int K,
                                                        int64_t step, int64_t ns, Elem* out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ns) return;
  const int r = find_slot(soff, K, g);
  out[g] = cur[eoff[r] + (g - soff[r]) * step + step / 2];
}

// bounds[j] = merged[(j + 1) * ns / C], j < C - 1
__global__ void __launch_bounds__(256) gk_pick_kernel(const Elem* merged, int64_t ns, int64_t C, Elem* bounds) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= C - 1) return;
  int64_t i = (j + 1) * ns / C;
  if (i > ns - 1) i = ns - 1;
  bounds[j] = merged[i];
}

// Position of every splitter among each run's samples without a search: splitter j is merged
// sample idx_j = (j + 1) * ns / C, so the run-r samples below it are the run-r samples among
// merged[0, idx_j). gk_hist_kernel buckets each merged sample by the first splitter above it
// (hist[r][b]); gk_hist_scan_kernel turns the histogram of each run into inclusive prefix counts.
// ord_off: run boundaries in record ordinals (the level-0 element offsets): an element's run is
// found from its ordinal at every recursion level, since level d's runs hold samples of run k only.
__global__ void __launch_bounds__(256) gk_hist_kernel(const Elem* merged, int64_t ns, int64_t C,
                                                      const int64_t* ord_off, int K, int* hist) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ns) return;
  int64_t b = i * C / ns;
  b = b > 0 ? b - 1 : 0;
  while (b < C - 1 && min((b + 1) * ns / C, ns - 1) <= i) ++b;  // first splitter index above i (C-1: none)
  if (b >= C - 1) return;
  const int r = find_slot(ord_off, K, (int64_t)(merged[i].lo & kGenOrdMask));
  atomicAdd(&hist[(int64_t)r * C + b], 1);
}

__global__ void __launch_bounds__(256) gk_hist_scan_kernel(int* hist, int64_t C) {
  __shared__ int part[256];
  int* h = hist + (int64_t)blockIdx.x * C;
  int carry = 0;
  for (int64_t base = 0; base < C; base += 256) {
    const int64_t j = base + threadIdx.x;
    const int v = j < C ? h[j] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // inclusive Hillis-Steele scan
      const int y = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
      __syncthreads();
      part[threadIdx.x] += y;
      __syncthreads();
    }
    if (j < C) h[j] = carry + part[threadIdx.x];
    carry += part[255];
    __syncthreads();
  }
}

// split[r * (C + 1) + j] from the prefix counts: the first run-r sample not below splitter j - 1 is
// sample cnt = hist[r][j - 1], so the answer lies in (pos(cnt - 1), pos(cnt)]: ~log2(step) probes.
__global__ void __launch_bounds__(256) gk_split_hist_kernel(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff,
                                                            const int64_t* soff, int64_t step, int K, const Elem* bounds,
                                                            int64_t C, const int* hist, int64_t* split) {
  // lanes of a wave take consecutive runs for the same splitter: the splitter's key bytes, read on
  // every prefix tie, are then one broadcast load instead of 64 scattered ones
  const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (int64_t)K * (C + 1)) return;
  const int r = (int)(u % K);
  const int64_t j = u / K;
  const int64_t t = (int64_t)r * (C + 1) + j;
  const int64_t n = eoff[r + 1] - eoff[r];
  if (j == 0 || j == C) {
    split[t] = j == 0 ? 0 : n;
    return;
  }
  const Elem b = bounds[j - 1];
  const int64_t ns = soff[r + 1] - soff[r];
  const int64_t cnt = min(max((int64_t)hist[(int64_t)r * C + (j - 1)], (int64_t)0), ns);
  int64_t a = cnt > 0 ? min((cnt - 1) * step + step / 2 + 1, n) : 0;
  int64_t z = cnt < ns ? min(cnt * step + step / 2, n) : n;
  const Elem* run = cur + eoff[r];
  while (a < z) {
    const int64_t mid = (a + z) >> 1;
    if (generic_lt(ctx, run[mid], b))
      a = mid + 1;
    else
      z = mid;
  }
  split[t] = a;
}

// Output rounds over cell ranges: for round boundary q at cell cb[q], elem[q] = sum over runs of
// the run's split there (merged elements before the boundary) and byte[q] = the record bytes before
// it (the F1 record offsets at the split). One block per boundary.
__global__ void __launch_bounds__(128) gk_round_bounds_kernel(const int64_t* split, int K, int64_t C, const int64_t* cb,
                                                              const int64_t* const* rec_off, int64_t* elem,
                                                              int64_t* bytes) {
  __shared__ unsigned long long se[128], sb[128];
  const int64_t c = cb[blockIdx.x];
  unsigned long long e = 0, b = 0;
  for (int k = threadIdx.x; k < K; k += 128) {
    const int64_t x = split[(int64_t)k * (C + 1) + c];
    e += (unsigned long long)x;
    b += (unsigned long long)rec_off[k][x];
  }
  se[threadIdx.x] = e;
  sb[threadIdx.x] = b;
  __syncthreads();
  for (int off = 64; off >= 1; off >>= 1) {
    if ((int)threadIdx.x < off) {
      se[threadIdx.x] += se[threadIdx.x + off];
      sb[threadIdx.x] += sb[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    elem[blockIdx.x] = (int64_t)se[0];
    bytes[blockIdx.x] = (int64_t)sb[0];
  }
}

__global__ void __launch_bounds__(kGkThreads) gk_cell_kernel(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff,
                                                             int K, const int64_t* split, int64_t C, int64_t c_first,
                                                             Elem* out, int* overflow) {
  __shared__ __attribute__((aligned(16))) Elem E[kGkCap];
  __shared__ uint64_t w0[kGkCap], w1[kGkCap], w2[kGkCap];
  __shared__ int32_t klen[kGkCap];
  __shared__ uint16_t ia[kGkCap], ib[kGkCap];
  __shared__ int seg[kGkMaxRuns + 1];
  __shared__ int64_t beg[kGkMaxRuns];
  __shared__ int64_t s_start;
  __shared__ int s_p, s_bad;
  const int64_t c = c_first + blockIdx.x;
  const int lane = threadIdx.x & 63;
  // ---- slices of this cell (wave 0): lengths scanned into seg, global start of each slice
  if (threadIdx.x < 64) {
    int carry = 0;
    unsigned long long bsum = 0;
    bool bad = false;
    if (lane == 0) seg[0] = 0;
    for (int base = 0; base < K; base += 64) {
      const int k = base + lane;
      int len = 0;
      if (k < K) {
        const int64_t b = split[(int64_t)k * (C + 1) + c], e = split[(int64_t)k * (C + 1) + c + 1];
        if (b < 0 || e < b || e > eoff[k + 1] - eoff[k] || e - b > kGkCap) bad = true;  // never read outside the run
        beg[k] = eoff[k] + b;
        len = bad ? 0 : (int)(e - b);
        bsum += (unsigned long long)b;
      }
      int x = len;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (k < K) seg[k + 1] = carry + x;
      carry += __shfl(x, 63, 64);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) bsum += __shfl_xor(bsum, off, 64);
    const bool any_bad = __any(bad);
    if (lane == 0) {
      s_start = (int64_t)bsum;
      s_bad = any_bad ? 1 : 0;
    }
  }
  __syncthreads();
  const int n = seg[K];
  if (n > kGkCap || s_bad) {  // uniform; cannot happen with the sampling bound and exact splits
    if (threadIdx.x == 0) atomicAdd(overflow, 1);
    return;
  }
  if (n == 0) return;
  // ---- elements into LDS (all of a thread's loads in flight)
  {
    Elem v[kGkItems];
#pragma unroll
    for (int k = 0; k < kGkItems; ++k) {
      const int i = min((int)threadIdx.x + k * kGkThreads, n - 1);
      int sl = 0, sh = K;
      while (sh - sl > 1) {
        const int mid = (sl + sh) >> 1;
        if (seg[mid] <= i)
          sl = mid;
        else
          sh = mid;
      }
      v[k] = cur[beg[sl] + (i - seg[sl])];
    }
#pragma unroll
    for (int k = 0; k < kGkItems; ++k) {
      const int i = threadIdx.x + k * kGkThreads;
      if (i < n) {
        E[i] = v[k];
        ia[i] = (uint16_t)i;
      }
    }
  }
  __syncthreads();
  // ---- P = LCP of the cell's keys = min over the slice end points of their LCP with E[0]
  if (threadIdx.x < 64) {
    const uint64_t g0 = E[0].lo & kGenOrdMask;
    const uint8_t* k0 = ctx.keyptr[g0];
    const int l0 = ctx.keylen[g0];
    int p = l0;
    for (int k = lane; k < K; k += 64) {
      if (seg[k + 1] > seg[k]) {
        const uint64_t ga = E[seg[k]].lo & kGenOrdMask, gz = E[seg[k + 1] - 1].lo & kGenOrdMask;
        p = key_lcp(k0, l0, ctx.keyptr[ga], ctx.keylen[ga], p);
        p = key_lcp(k0, l0, ctx.keyptr[gz], ctx.keylen[gz], p);
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p = min(p, __shfl_xor(p, off, 64));
    if (lane == 0) s_p = p;
  }
  __syncthreads();
  const int P = s_p;
  // ---- stage key bytes [P, P + 24) of every element
  for (int i = threadIdx.x; i < n; i += kGkThreads) {
    const uint64_t g = E[i].lo & kGenOrdMask;
    const uint8_t* kp = ctx.keyptr[g];
    const int l = ctx.keylen[g];
    const int rem = l - P;
    klen[i] = l;
    w0[i] = rem > 0 ? load_be8(kp + P, rem) : 0;
    w1[i] = rem > 8 ? load_be8(kp + P + 8, rem - 8) : 0;
    w2[i] = rem > 16 ? load_be8(kp + P + 16, rem - 16) : 0;
  }
  __syncthreads();
  auto le = [&](int x, int y) -> bool {
    if (w0[x] != w0[y]) return w0[x] < w0[y];
    if (w1[x] != w1[y]) return w1[x] < w1[y];
    if (w2[x] != w2[y]) return w2[x] < w2[y];
    const int lx = klen[x], ly = klen[y];
    if (lx > P + 24 && ly > P + 24) {
      const uint8_t* px = ctx.keyptr[E[x].lo & kGenOrdMask];
      const uint8_t* py = ctx.keyptr[E[y].lo & kGenOrdMask];
      const int m = lx < ly ? lx : ly;
      for (int i = P + 24; i < m; i += 8) {
        const uint64_t a = load_be8(px + i, m - i), b = load_be8(py + i, m - i);
        if (a != b) return a < b;
      }
    }
    if (lx != ly) return lx < ly;
    return (E[x].lo & kGenOrdMask) <= (E[y].lo & kGenOrdMask);
  };
  // ---- pairwise merge levels on element indices
  uint16_t* src = ia;
  uint16_t* dst = ib;
  const int o0 = threadIdx.x * kGkItems;
  for (int w = 1; w < K; w <<= 1) {
    if (o0 < n) {
      const int npairs = (K + 2 * w - 1) / (2 * w);
      int pl = 0, ph = npairs;
      while (ph - pl > 1) {
        const int mid = (pl + ph) >> 1;
        if (seg[min(2 * mid * w, K)] <= o0)
          pl = mid;
        else
          ph = mid;
      }
      int p = pl;
      int a0 = seg[min(2 * p * w, K)], a1 = seg[min((2 * p + 1) * w, K)], b1 = seg[min((2 * p + 2) * w, K)];
      int d = o0 - a0, la = a1 - a0, lb = b1 - a1;
      int ml = d > lb ? d - lb : 0, mh = d < la ? d : la;
      while (ml < mh) {
        const int mid = (ml + mh) >> 1;
        if (le(src[a0 + mid], src[a1 + d - 1 - mid]))
          ml = mid + 1;
        else
          mh = mid;
      }
      int xa = ml, xb = d - ml;
      const int todo = min(kGkItems, n - o0);
      for (int k = 0; k < todo; ++k) {
        const int o = o0 + k;
        while (o == b1) {  // next pair (empty pairs are skipped)
          ++p;
          a0 = b1;
          a1 = seg[min((2 * p + 1) * w, K)];
          b1 = seg[min((2 * p + 2) * w, K)];
          la = a1 - a0;
          lb = b1 - a1;
          xa = 0;
          xb = 0;
        }
        const bool take_a = xb >= lb || (xa < la && le(src[a0 + xa], src[a1 + xb]));
        dst[o] = take_a ? src[a0 + xa] : src[a1 + xb];
        if (take_a)
          ++xa;
        else
          ++xb;
      }
    }
    __syncthreads();
    uint16_t* t = src;
    src = dst;
    dst = t;
  }
  // ---- merged elements out
  Elem* o = out + s_start;
  for (int i = threadIdx.x; i < n; i += kGkThreads) o[i] = E[src[i]];
}

}  // namespace

int generic_kway_cap() { return kGkCap; }

void launch_gk_sample(const Elem* cur, const int64_t* eoff, const int64_t* soff, int K, int64_t step, int64_t ns,
                      Elem* out, hipStream_t s) {
  if (ns <= 0) return;
  hipLaunchKernelGGL(gk_sample_kernel, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, cur, eoff, soff, K, step,
                     ns, out);
}

void launch_gk_pick(const Elem* merged, int64_t ns, int64_t C, Elem* bounds, hipStream_t s) {
  if (C <= 1) return;
  hipLaunchKernelGGL(gk_pick_kernel, dim3((unsigned)((C - 1 + 255) / 256)), dim3(256), 0, s, merged, ns, C, bounds);
}

void launch_gk_split_hist(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff, const int64_t* ord_off,
                          const Elem* merged, int64_t ns, const int64_t* soff, int64_t step, int K, const Elem* bounds,
                          int64_t C, int* hist, int64_t* split, hipStream_t s) {
  if (C > 1 && ns > 0) {
    (void)hipMemsetAsync(hist, 0, sizeof(int) * (size_t)K * (size_t)C, s);
    hipLaunchKernelGGL(gk_hist_kernel, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, merged, ns, C, ord_off,
                       K, hist);
    hipLaunchKernelGGL(gk_hist_scan_kernel, dim3((unsigned)K), dim3(256), 0, s, hist, C);
  }
  const int64_t n = (int64_t)K * (C + 1);
  hipLaunchKernelGGL(gk_split_hist_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ctx, cur, eoff, soff,
                     step, K, bounds, C, hist, split);
}

void launch_gk_cells(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff, int K, const int64_t* split, int64_t C,
                     int64_t c_first, int64_t c_count, Elem* out, int* overflow, hipStream_t s) {
  if (c_count <= 0) return;
  hipLaunchKernelGGL(gk_cell_kernel, dim3((unsigned)c_count), dim3(kGkThreads), 0, s, ctx, cur, eoff, K, split, C,
                     c_first, out, overflow);
}

void launch_gk_round_bounds(const int64_t* split, int K, int64_t C, const int64_t* cb, int nb,
                            const int64_t* const* rec_off, int64_t* elem, int64_t* bytes, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(gk_round_bounds_kernel, dim3((unsigned)nb), dim3(128), 0, s, split, K, C, cb, rec_off, elem,
                     bytes);
}

}  // namespace gpu
}  // namespace uda
