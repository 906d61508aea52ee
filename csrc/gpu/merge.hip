// K-way merge of sorted runs on gfx950: key extraction (F2), merge-path merge tree (F3),
// record gather/serialize (F4) and device-side validation.
//
// Reference hot loop replaced: PriorityQueue::downHeap + MergeQueue::next/adjustPriorityQueue
// (src/Merger/MergeQueue.h:250-269, 299-321, 390-419) driving BaseSegment::nextKVInternal
// (src/Merger/StreamRW.cc:334-404) and write_kv_to_stream (StreamRW.cc:151-225): one comparator
// call per heap level per record on one CPU thread.
//
// MI355X design:
//  * F2: every record's key becomes one 16-byte integer element (Elem) in a compact array, so the
//    merge moves 16 B per record per level instead of touching 104-byte records.
//  * F3: ceil(log2 K) pairwise merge-path passes. Each pass is split into 2048-element output tiles
//    (one 256-thread workgroup each, 8 elements per lane); tile boundaries are found by a separate
//    partition kernel (one lane per tile, binary search along the cross diagonal), then each
//    workgroup stages its A and B slices in LDS (32 KiB), merges lane-locally after an LDS
//    merge-path search, re-stages the merged tile in LDS and writes it out fully coalesced.
//    Exact split points make every tile exactly 2048 elements regardless of key skew or duplicates.
//  * F4: one final gather moves each 104-byte record once: a wave owns 64 consecutive output
//    records and streams them as 832 consecutive 8-byte words (13 per record), so every store
//    instruction writes 512 contiguous bytes and every load reads whole record spans.
#include "generic_cmp.h"
#include "kernels.h"
#include "uda/compare.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {

__device__ __forceinline__ bool elem_le(const Elem& a, const Elem& b) {
  return a.hi < b.hi || (a.hi == b.hi && a.lo <= b.lo);
}

// FIXED10: (hi, lo) is the whole key plus the (run, pos) tie-break.
struct FixedCmp {
  __device__ __forceinline__ bool le(const Elem& a, const Elem& b) const { return elem_le(a, b); }
};

// GENERIC: the total order of generic_cmp.h.
struct GenericCmp {
  GenericKeyCtx ctx;
  __device__ __forceinline__ bool le(const Elem& a, const Elem& b) const { return generic_le(ctx, a, b); }
};

__device__ __forceinline__ Elem ld_elem(const Elem* p) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  Elem e;
  e.hi = (uint64_t)v.x | ((uint64_t)v.y << 32);
  e.lo = (uint64_t)v.z | ((uint64_t)v.w << 32);
  return e;
}

__device__ __forceinline__ void st_elem(Elem* p, const Elem& e) {
  uint4 v;
  v.x = (uint32_t)e.hi;
  v.y = (uint32_t)(e.hi >> 32);
  v.z = (uint32_t)e.lo;
  v.w = (uint32_t)(e.lo >> 32);
  *reinterpret_cast<uint4*>(p) = v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ------------------------------------------------------------------------- F2: key extraction
__global__ void __launch_bounds__(256) extract_fixed_kernel(const RunDesc* runs,
                                                            const int64_t* elem_off, int nruns,
                                                            int64_t total, Elem* out,
                                                            int* bad_layout) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  // locate the run: elem_off is ascending with nruns+1 entries
  int lo = 0, hi = nruns;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (elem_off[mid] <= g)
      lo = mid;
    else
      hi = mid;
  }
  const int r = lo;
  const int64_t pos = g - elem_off[r];
  const uint8_t* rec = runs[r].base + pos * kTeraRecordBytes;
  const uint64_t w0 = *reinterpret_cast<const uint64_t*>(rec);
  const uint64_t w1 = *reinterpret_cast<const uint64_t*>(rec + 8);
  // header: keyLen VInt 11, valLen VInt 91, Text VInt 10, value Text VInt 90 at byte 13
  if ((w0 & 0xFFFFFF) != 0x0A5B0B || ((w1 >> 40) & 0xFF) != 0x5A) *bad_layout = 1;
  const uint64_t b0 = __builtin_bswap64(w0), b1 = __builtin_bswap64(w1);
  Elem e;
  e.hi = (b0 << 24) | (b1 >> 40);
  e.lo = (((b1 >> 24) & 0xFFFF) << 48) | ((uint64_t)r << 32) | (uint64_t)pos;
  st_elem(out + g, e);
}

// ------------------------------------------------------------------------- F3: merge path
template <class Cmp>
__device__ __forceinline__ int64_t merge_path_global(const Cmp& cmp, const Elem* A, int64_t a_len, const Elem* B,
                                                     int64_t b_len, int64_t diag) {
  int64_t lo = diag > b_len ? diag - b_len : 0;
  int64_t hi = diag < a_len ? diag : a_len;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (cmp.le(ld_elem(A + mid), ld_elem(B + (diag - 1 - mid))))
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// Resolve tile t of a pass to its pair geometry.
struct TileGeo {
  int64_t a0, a_len, b_len, d0;
  int pair;
};
template <int TILE>
__device__ __forceinline__ TileGeo tile_geo(const PassDesc& pd, int t) {
  int lo = 0, hi = pd.npairs;  // tile_prefix[lo] <= t < tile_prefix[lo+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pd.tile_prefix[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  TileGeo g;
  g.pair = lo;
  g.a0 = pd.pairs[3 * lo];
  g.a_len = pd.pairs[3 * lo + 1] - g.a0;
  g.b_len = pd.pairs[3 * lo + 2] - pd.pairs[3 * lo + 1];
  g.d0 = (int64_t)(t - pd.tile_prefix[lo]) * TILE;
  return g;
}

template <int TILE, class Cmp>
__global__ void __launch_bounds__(256) merge_partition_kernel(const Elem* in, PassDesc pd,
                                                              int64_t* splits, Cmp cmp) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= pd.ntiles) return;
  const TileGeo g = tile_geo<TILE>(pd, t);
  const Elem* A = in + g.a0;
  splits[t] = merge_path_global(cmp, A, g.a_len, A + g.a_len, g.b_len, g.d0);
}

constexpr int kThreads = 256;
constexpr int kItems = kMergeTile / kThreads;  // 8

template <class Cmp>
__global__ void __launch_bounds__(kThreads) merge_pass_kernel(const Elem* in, Elem* out, PassDesc pd,
                                                              const int64_t* splits, Cmp cmp) {
  __shared__ __attribute__((aligned(16))) Elem lds[kMergeTile];
  const int t = blockIdx.x;
  const TileGeo g = tile_geo<kMergeTile>(pd, t);
  const int64_t pair_len = g.a_len + g.b_len;
  const int64_t d0 = g.d0;
  const int64_t d1 = (d0 + kMergeTile < pair_len) ? d0 + kMergeTile : pair_len;
  const int64_t i0 = splits[t];
  const bool last_of_pair = (t + 1 >= (int)pd.tile_prefix[g.pair + 1]);
  const int64_t i1 = last_of_pair ? g.a_len : splits[t + 1];
  const int cnt = (int)(d1 - d0);
  const int la = (int)(i1 - i0);
  const int lb = cnt - la;
  const Elem* A = in + g.a0 + i0;
  const Elem* B = in + g.a0 + g.a_len + (d0 - i0);

  // Stage A-slice then B-slice contiguously in LDS (coalesced 16-byte loads).
  for (int k = threadIdx.x; k < cnt; k += kThreads) {
    const Elem e = (k < la) ? ld_elem(A + k) : ld_elem(B + (k - la));
    st_elem(lds + k, e);
  }
  __syncthreads();

  // Lane-local merge of up to kItems outputs starting at diagonal tid*kItems. Results stay in
  // registers (split hi/lo arrays, fully unrolled: no scratch) until the tile is re-staged.
  const int diag = threadIdx.x * kItems;
  uint64_t rh[kItems], rl[kItems];
  int todo = 0;
  if (diag < cnt) {
    int lo = diag > lb ? diag - lb : 0;
    int hi = diag < la ? diag : la;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cmp.le(lds[mid], lds[la + diag - 1 - mid]))
        lo = mid + 1;
      else
        hi = mid;
    }
    int ia = lo, ib = diag - lo;
    todo = (cnt - diag) < kItems ? (cnt - diag) : kItems;
    Elem ea = (ia < la) ? lds[ia] : Elem{~0ull, ~0ull};
    Elem eb = (ib < lb) ? lds[la + ib] : Elem{~0ull, ~0ull};
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const bool take_a = (ib >= lb) || (ia < la && cmp.le(ea, eb));
      rh[k] = take_a ? ea.hi : eb.hi;
      rl[k] = take_a ? ea.lo : eb.lo;
      if (take_a) {
        ++ia;
        ea = (ia < la) ? lds[ia] : Elem{~0ull, ~0ull};
      } else {
        ++ib;
        eb = (ib < lb) ? lds[la + ib] : Elem{~0ull, ~0ull};
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kItems; ++k)
    if (k < todo) st_elem(lds + diag + k, Elem{rh[k], rl[k]});
  __syncthreads();
  Elem* O = out + g.a0 + d0;
  for (int k = threadIdx.x; k < cnt; k += kThreads) st_elem(O + k, lds[k]);
}

// GENERIC merge pass with LDS-staged key bytes. Every key of a tile lies between the first and last
// element of its A and B slices (both sorted), so the longest common prefix P of those four keys is a
// prefix of every key in the tile. Each element's key bytes [P, P+24) are staged in LDS once (three
// big-endian words, zero padded past the key end); comparisons then run on LDS words and reach HBM
// only for keys that still tie after P+24 bytes. Order = content bytes, then length, then ordinal:
// the same total order as GenericCmp (used by the partition kernel).
constexpr int kGenItems = kGenericMergeTile / kThreads;  // 4
constexpr uint64_t kOrdMask = kGenOrdMask;

__global__ void __launch_bounds__(kThreads) merge_pass_generic_lds_kernel(const Elem* in, Elem* out, PassDesc pd,
                                                                          const int64_t* splits, GenericKeyCtx ctx) {
  constexpr int TILE = kGenericMergeTile;
  __shared__ __attribute__((aligned(16))) Elem lds[TILE];
  __shared__ uint64_t w0[TILE], w1[TILE], w2[TILE];
  __shared__ int32_t klen[TILE];
  __shared__ int tile_p;
  const int t = blockIdx.x;
  const TileGeo g = tile_geo<TILE>(pd, t);
  const int64_t pair_len = g.a_len + g.b_len;
  const int64_t d0 = g.d0;
  const int64_t d1 = (d0 + TILE < pair_len) ? d0 + TILE : pair_len;
  const int64_t i0 = splits[t];
  const bool last_of_pair = (t + 1 >= (int)pd.tile_prefix[g.pair + 1]);
  const int64_t i1 = last_of_pair ? g.a_len : splits[t + 1];
  const int cnt = (int)(d1 - d0);
  const int la = (int)(i1 - i0);
  const int lb = cnt - la;
  const Elem* A = in + g.a0 + i0;
  const Elem* B = in + g.a0 + g.a_len + (d0 - i0);
  for (int k = threadIdx.x; k < cnt; k += kThreads) {
    const Elem e = (k < la) ? ld_elem(A + k) : ld_elem(B + (k - la));
    st_elem(lds + k, e);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int ends[4], ne = 0;
    if (la > 0) { ends[ne++] = 0; ends[ne++] = la - 1; }
    if (lb > 0) { ends[ne++] = la; ends[ne++] = cnt - 1; }
    int p = 1 << 30;
    if (ne > 0) {
      const uint64_t g0 = lds[ends[0]].lo & kOrdMask;
      const uint8_t* k0 = ctx.keyptr[g0];
      const int l0 = ctx.keylen[g0];
      p = l0;
      for (int x = 1; x < ne; ++x) {
        const uint64_t gx = lds[ends[x]].lo & kOrdMask;
        p = key_lcp(k0, l0, ctx.keyptr[gx], ctx.keylen[gx], p);
      }
    }
    tile_p = (ne > 0) ? p : 0;
  }
  __syncthreads();
  const int P = tile_p;
  for (int k = threadIdx.x; k < cnt; k += kThreads) {
    const uint64_t gk = lds[k].lo & kOrdMask;
    const uint8_t* kp = ctx.keyptr[gk];
    const int l = ctx.keylen[gk];
    klen[k] = l;
    const int rem = l - P;
    w0[k] = rem > 0 ? load_be8(kp + P, rem) : 0;
    w1[k] = rem > 8 ? load_be8(kp + P + 8, rem - 8) : 0;
    w2[k] = rem > 16 ? load_be8(kp + P + 16, rem - 16) : 0;
  }
  __syncthreads();
  auto le = [&](int x, int y) -> bool {
    if (w0[x] != w0[y]) return w0[x] < w0[y];
    if (w1[x] != w1[y]) return w1[x] < w1[y];
    if (w2[x] != w2[y]) return w2[x] < w2[y];
    const int lx = klen[x], ly = klen[y];
    if (lx > P + 24 && ly > P + 24) {
      const uint8_t* px = ctx.keyptr[lds[x].lo & kOrdMask];
      const uint8_t* py = ctx.keyptr[lds[y].lo & kOrdMask];
      const int n = lx < ly ? lx : ly;
      for (int i = P + 24; i < n; i += 8) {
        const uint64_t a = load_be8(px + i, n - i), b = load_be8(py + i, n - i);
        if (a != b) return a < b;
      }
    }
    if (lx != ly) return lx < ly;
    return (lds[x].lo & kOrdMask) <= (lds[y].lo & kOrdMask);
  };
  const int diag = threadIdx.x * kGenItems;
  int res[kGenItems];
  int todo = 0;
  if (diag < cnt) {
    int lo = diag > lb ? diag - lb : 0;
    int hi = diag < la ? diag : la;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (le(mid, la + diag - 1 - mid))
        lo = mid + 1;
      else
        hi = mid;
    }
    int ia = lo, ib = diag - lo;
    todo = (cnt - diag) < kGenItems ? (cnt - diag) : kGenItems;
#pragma unroll
    for (int k = 0; k < kGenItems; ++k) {
      const bool take_a = (ib >= lb) || (ia < la && le(ia, la + ib));
      res[k] = take_a ? ia : la + ib;
      if (take_a)
        ++ia;
      else
        ++ib;
    }
  }
  Elem r[kGenItems];
#pragma unroll
  for (int k = 0; k < kGenItems; ++k)
    if (k < todo) r[k] = lds[res[k]];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kGenItems; ++k)
    if (k < todo) st_elem(lds + diag + k, r[k]);
  __syncthreads();
  Elem* O = out + g.a0 + d0;
  for (int k = threadIdx.x; k < cnt; k += kThreads) st_elem(O + k, lds[k]);
}

// ------------------------------------------------------------------------- F4: gather
// One wave per 64 consecutive output records; 13 passes of 64 x 8-byte words.
__global__ void __launch_bounds__(256) gather_fixed_kernel(const Elem* elems, int64_t n,
                                                           uint8_t* const* run_bases,
                                                           uint8_t* out) {
  constexpr int kWords = kTeraRecordBytes / 8;  // 13
  const int lane = threadIdx.x & 63;
  const int64_t rec0 =
      ((int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 64;  // wave-uniform
  if (rec0 >= n) return;
  const int valid = (n - rec0) < 64 ? (int)(n - rec0) : 64;
  unsigned long long src = 0;
  if (lane < valid) {
    const Elem e = ld_elem(elems + rec0 + lane);
    const int run = (int)((e.lo >> 32) & 0xFFFF);
    const uint64_t pos = e.lo & 0xFFFFFFFFull;
    src = (unsigned long long)(run_bases[run] + pos * kTeraRecordBytes);
  }
  uint64_t* dst = reinterpret_cast<uint64_t*>(out + rec0 * kTeraRecordBytes);
  // every load of the lane before its first store (a load -> store chain serializes on aliasing),
  // and no per-lane guards on full waves (guarded stores each drain vmcnt)
  uint64_t v[kWords];
  if (valid == 64) {
#pragma unroll
    for (int j = 0; j < kWords; ++j) {
      const int w = j * 64 + lane;
      const int r = w / kWords;
      v[j] = ((const __attribute__((address_space(1))) uint64_t*)__shfl(src, r, 64))[w - r * kWords];
    }
#pragma unroll
    for (int j = 0; j < kWords; ++j) dst[j * 64 + lane] = v[j];
    return;
  }
  const int words = valid * kWords;
#pragma unroll
  for (int j = 0; j < kWords; ++j) {
    const int w = j * 64 + lane;
    const int r = w / kWords;
    const unsigned long long s = __shfl(src, r < 64 ? r : 63, 64);
    v[j] = w < words ? reinterpret_cast<const uint64_t*>(s)[w - r * kWords] : 0;
  }
#pragma unroll
  for (int j = 0; j < kWords; ++j) {
    const int w = j * 64 + lane;
    if (w < words) dst[w] = v[j];
  }
}

// ------------------------------------------------------------------------- validation
__global__ void __launch_bounds__(256) validate_fixed_kernel(const uint8_t* recs, int64_t n,
                                                             const Elem* prev_key, int has_prev,
                                                             Elem* last_key,
                                                             unsigned long long* stats,
                                                             unsigned long long* group_ck) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long bad = 0, h = 0;
  if (i < n) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(recs + i * kTeraRecordBytes);
    uint64_t hh = 0x9E3779B97F4A7C15ULL ^ (uint64_t)kTeraRecordBytes;
#pragma unroll
    for (int j = 0; j < 13; ++j) hh = mix64(hh ^ w[j]);
    h = hh;
    const uint64_t b0 = __builtin_bswap64(w[0]), b1 = __builtin_bswap64(w[1]);
    const uint64_t khi = (b0 << 24) | (b1 >> 40), klo = (b1 >> 24) & 0xFFFF;
    if (i + 1 < n) {
      const uint64_t* v = reinterpret_cast<const uint64_t*>(recs + (i + 1) * kTeraRecordBytes);
      const uint64_t c0 = __builtin_bswap64(v[0]), c1 = __builtin_bswap64(v[1]);
      const uint64_t nhi = (c0 << 24) | (c1 >> 40), nlo = (c1 >> 24) & 0xFFFF;
      if (khi > nhi || (khi == nhi && klo > nlo)) bad = 1;
    } else {
      last_key->hi = khi;
      last_key->lo = klo << 48;
    }
    if (i == 0 && has_prev) {
      const uint64_t phi = prev_key->hi, plo = prev_key->lo >> 48;
      if (phi > khi || (phi == khi && plo > klo)) bad += 1;
    }
  }
  bad = wave_sum_u64(bad);
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0) {
    if (bad) atomicAdd(stats + 0, bad);
    if (h) atomicAdd(stats + 1, h);
    if (h && group_ck) atomicAdd(group_ck, h);
  }
}

// Sum of record hashes of every FIXED10 slice (exchange verification): grid.y = slice.
__global__ void __launch_bounds__(256) slice_checksum_kernel(const RunDesc* runs, unsigned long long* out) {
  const RunDesc r = runs[blockIdx.y];
  unsigned long long h = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.nrec; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(r.base + i * kTeraRecordBytes);
    uint64_t hh = 0x9E3779B97F4A7C15ULL ^ (uint64_t)kTeraRecordBytes;
#pragma unroll
    for (int j = 0; j < 13; ++j) hh = mix64(hh ^ w[j]);
    h += hh;
  }
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0 && h) atomicAdd(out + blockIdx.y, h);
}

// FIXED10 layout check of every record of every run: grid.y = run.
__global__ void __launch_bounds__(256) check_fixed_kernel(const RunDesc* runs, int* bad) {
  const RunDesc r = runs[blockIdx.y];
  int b = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.nrec; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* rec = r.base + i * kTeraRecordBytes;
    const uint64_t w0 = *reinterpret_cast<const uint64_t*>(rec);
    const uint64_t w1 = *reinterpret_cast<const uint64_t*>(rec + 8);
    if ((w0 & 0xFFFFFF) != 0x0A5B0B || ((w1 >> 40) & 0xFF) != 0x5A) b = 1;
  }
  if (b) *bad = 1;
}

__global__ void __launch_bounds__(256) count_mismatch_kernel(const unsigned long long* a,
                                                             const unsigned long long* b, int n,
                                                             unsigned long long* errors) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && a[i] != b[i]) atomicAdd(errors, 1ull);
}

}  // namespace

void launch_extract_fixed(const RunDesc* runs, const int64_t* elem_off, int nruns, int64_t total,
                          Elem* out, int* bad_layout, hipStream_t s) {
  if (total <= 0) return;
  hipLaunchKernelGGL(extract_fixed_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     runs, elem_off, nruns, total, out, bad_layout);
}

void launch_merge_partition(const Elem* in, PassDesc pd, int64_t* splits, hipStream_t s) {
  if (pd.ntiles <= 0) return;
  hipLaunchKernelGGL((merge_partition_kernel<kMergeTile, FixedCmp>), dim3((unsigned)((pd.ntiles + 255) / 256)),
                     dim3(256), 0, s, in, pd, splits, FixedCmp{});
}

void launch_merge_pass(const Elem* in, Elem* out, PassDesc pd, const int64_t* splits,
                       hipStream_t s) {
  if (pd.ntiles <= 0) return;
  hipLaunchKernelGGL(merge_pass_kernel<FixedCmp>, dim3((unsigned)pd.ntiles), dim3(kThreads), 0, s, in, out,
                     pd, splits, FixedCmp{});
}

void launch_merge_partition_generic(const Elem* in, PassDesc pd, int64_t* splits, GenericKeyCtx ctx,
                                    hipStream_t s) {
  if (pd.ntiles <= 0) return;
  hipLaunchKernelGGL((merge_partition_kernel<kGenericMergeTile, GenericCmp>),
                     dim3((unsigned)((pd.ntiles + 255) / 256)), dim3(256), 0, s, in, pd, splits, GenericCmp{ctx});
}

void launch_merge_pass_generic(const Elem* in, Elem* out, PassDesc pd, const int64_t* splits,
                               GenericKeyCtx ctx, hipStream_t s) {
  if (pd.ntiles <= 0) return;
  hipLaunchKernelGGL(merge_pass_generic_lds_kernel, dim3((unsigned)pd.ntiles), dim3(kThreads), 0, s, in, out, pd,
                     splits, ctx);
}

void launch_gather_fixed(const Elem* elems, int64_t n, uint8_t* const* run_bases, uint8_t* out,
                         hipStream_t s) {
  if (n <= 0) return;
  const int64_t waves = (n + 63) / 64;
  hipLaunchKernelGGL(gather_fixed_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, elems,
                     n, run_bases, out);
}

void launch_validate_fixed(const uint8_t* recs, int64_t n, const Elem* prev_key, int has_prev,
                           Elem* last_key, unsigned long long* stats, hipStream_t s, unsigned long long* group_ck) {
  if (n <= 0) return;
  hipLaunchKernelGGL(validate_fixed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     recs, n, prev_key, has_prev, last_key, stats, group_ck);
}

}  // namespace gpu
}  // namespace uda

namespace uda {
namespace gpu {
void launch_slice_checksums(const RunDesc* runs, int n, int64_t max_nrec, unsigned long long* out, hipStream_t s) {
  if (n <= 0) return;
  (void)hipMemsetAsync(out, 0, sizeof(unsigned long long) * (size_t)n, s);
  int64_t bx = (max_nrec + 4095) / 4096;
  if (bx < 1) bx = 1;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(slice_checksum_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, s, runs, out);
}

void launch_count_mismatch(const unsigned long long* a, const unsigned long long* b, int n,
                           unsigned long long* errors, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(count_mismatch_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b, n, errors);
}
}  // namespace gpu
}  // namespace uda

namespace uda {
namespace gpu {
void launch_check_fixed(const RunDesc* runs, int n, int64_t max_nrec, int* bad, hipStream_t s) {
  if (n <= 0) return;
  int64_t bx = (max_nrec + 4095) / 4096;
  if (bx < 1) bx = 1;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(check_fixed_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, s, runs, bad);
}
}  // namespace gpu
}  // namespace uda
