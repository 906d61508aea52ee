// Single-pass K-way merge of FIXED10 (TeraSort) runs: F2 + F3 + F4 fused per output cell.
//
// Reference hot loop replaced: PriorityQueue::downHeap + MergeQueue::next/adjustPriorityQueue
// (src/Merger/MergeQueue.h:238-269, 299-321, 390-419) over all segments of a reduce task, and the
// record serialization behind it (write_kv_to_stream, src/Merger/StreamRW.cc:151-225).
//
// Design (gfx950):
//  * Cells by sampling. Every s-th key of every run is sampled; the samples of a group (reducer)
//    are merged and every (samples / cells)-th becomes a splitter; lower_bound of each splitter in
//    each run gives the cell slices. With s = (cap - T) / (K + 2) a cell holds at most
//    T + K*s <= cap records (T = target), so it always fits LDS; output offsets are the sums of the
//    lower bounds, no scan needed.
//  * One workgroup per cell (256 threads; cap = 2048 records by default, 512..2048 selectable,
//    cells planned to 65 % of it): the slices' keys are loaded once from the records into LDS as
//    16-byte elements (F2), the K sorted slices are merged pairwise inside LDS (log2 K levels, merge
//    path per thread over ceil(n / 256) outputs; by default every level is written back in place
//    into one cap x 16-byte buffer, two barriers per level, so 4 workgroups fit a CU; no HBM
//    traffic between levels), and the records are
//    gathered straight to the output (F4): one wave per 64 output records, 13 consecutive 8-byte
//    words per record, 512-byte coalesced stores. HBM traffic per record: its key line, then one
//    record read and one record write.
//  * The kernel is latency-bound (PMC: 66% of wave cycles waiting, HBM at ~3.5 TB/s read+write),
//    so every phase keeps its loads in flight together: F2 issues all of a thread's key loads
//    before the first LDS write, F4 all 13 word loads of a lane before its first store (with no
//    per-lane guards on full waves, which would split the stores into blocks that each drain
//    vmcnt). Round 2 ran 1536-record cells in two buffers (3 workgroups per CU, 51 KiB LDS each,
//    92 VGPRs); round 3's in-place levels and bigger, fuller cells are +18.5 % (device-only sweep,
//    profiles/r3_kway_occupancy.md). Per-phase timings come from UDA_KWAY_PROF.
//  * A cell that would not fit LDS (only possible with massively duplicated keys) is merged by a
//    wave-level priority queue: lanes own runs, a wave argmin picks the next record each step.
#include "kernels.h"

#include <mutex>
#include <stdexcept>
#include <string>

namespace uda {
namespace gpu {

namespace {

__device__ __forceinline__ bool kle(const Elem& a, const Elem& b) {
  return a.hi < b.hi || (a.hi == b.hi && a.lo <= b.lo);
}

typedef __attribute__((address_space(1))) const uint64_t GlobalU64;
typedef __attribute__((address_space(1))) const void GlobalVoid;
typedef __attribute__((address_space(3))) void LdsVoid;
// Run pointers are generic; the records live in global memory, so load through that address space.
__device__ __forceinline__ const GlobalU64* gptr(const void* p) { return (const GlobalU64*)(uintptr_t)p; }

__device__ __forceinline__ Elem key_elem(uint64_t w0, uint64_t w1, int run, int64_t pos, int& bad) {
  bad |= (w0 & 0xFFFFFF) != 0x0A5B0B || ((w1 >> 40) & 0xFF) != 0x5A;
  const uint64_t b0 = __builtin_bswap64(w0), b1 = __builtin_bswap64(w1);
  Elem e;
  e.hi = (b0 << 24) | (b1 >> 40);
  e.lo = (((b1 >> 24) & 0xFFFF) << 48) | ((uint64_t)run << 32) | (uint64_t)pos;
  return e;
}

__device__ __forceinline__ Elem load_key_elem(const uint8_t* rec, int run, int64_t pos, int* bad) {
  const GlobalU64* w = gptr(rec);
  int b = 0;
  const Elem e = key_elem(w[0], w[1], run, pos, b);
  if (b) *bad = 1;
  return e;
}

__global__ void __launch_bounds__(256) pick_splitters_kernel(const Elem* samples, const int64_t* gsamp_off,
                                                             const int64_t* gcells, int G, int nbmax, Elem* bounds) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)G * nbmax) return;
  const int g = (int)(t / nbmax), j = (int)(t % nbmax);
  const int64_t C = gcells[g];
  const int64_t ns = gsamp_off[g + 1] - gsamp_off[g];
  Elem b{~0ull, ~0ull};
  if (j < C - 1 && ns > 0) {
    int64_t idx = (int64_t)(j + 1) * ns / C;
    if (idx > ns - 1) idx = ns - 1;
    const Elem s = samples[gsamp_off[g] + idx];
    b.hi = s.hi;
    b.lo = s.lo & (0xFFFFull << 48);
  }
  bounds[t] = b;
}

// Cell split points: split[r][c] = first record of run r with key >= splitter c-1 of its group. The
// run's own regular sample (sample j = record j*every + every/2, sorted like the run) brackets the
// answer first, so only ~log2(every) probes touch the 104-byte records; the dense 16-byte samples
// stay in L2. (A plain binary search over the run costs ~log2(nrec) scattered record lines.)
__global__ void __launch_bounds__(256) split_sampled_kernel(uint8_t* const* bases, const int64_t* nrec,
                                                            const Elem* samples, const int64_t* soff, int64_t every,
                                                            const Elem* bounds, const int* run_bound_set, int nruns,
                                                            int nb, int64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t per = nb + 2;
  if (t >= (int64_t)nruns * per) return;
  const int r = (int)(t / per);
  const int b = (int)(t % per);
  const int64_t n = nrec[r];
  if (b == 0 || b == nb + 1) {
    out[t] = b == 0 ? 0 : n;
    return;
  }
  const Elem bound = bounds[(int64_t)run_bound_set[r] * nb + (b - 1)];
  const uint64_t btail = bound.lo >> 48;
  // first sample with key >= bound
  const Elem* smp = samples + soff[r];
  int64_t lo = 0, hi = soff[r + 1] - soff[r];
  const int64_t ns = hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const Elem e = smp[mid];
    if (e.hi < bound.hi || (e.hi == bound.hi && (e.lo >> 48) < btail))
      lo = mid + 1;
    else
      hi = mid;
  }
  // samples lo-1 < bound <= sample lo: the answer lies in (pos(lo-1), pos(lo)]
  int64_t a = lo > 0 ? (lo - 1) * every + every / 2 + 1 : 0;
  int64_t z = lo < ns ? lo * every + every / 2 : n;
  if (z > n) z = n;
  const uint8_t* base = bases[r];
  while (a < z) {
    const int64_t mid = (a + z) >> 1;
    const GlobalU64* w = gptr(base + mid * kTeraRecordBytes);
    const uint64_t b0 = __builtin_bswap64(w[0]), b1 = __builtin_bswap64(w[1]);
    const uint64_t kh = (b0 << 24) | (b1 >> 40), kl = (b1 >> 24) & 0xFFFF;
    if (kh < bound.hi || (kh == bound.hi && kl < btail))
      a = mid + 1;
    else
      z = mid;
  }
  out[t] = a;
}

// Wave 0: exclusive scan of the K slice lengths into seg[0..K], each slice's first record into
// sbase[k], and the sum of the slice starts (the cell's first output record within its group).
__device__ __forceinline__ void kw_slices(const KwayDesc& kd, int c, int ncell, int r0, int K, int* seg,
                                          const uint8_t** sbase, int64_t* start_sum) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const int per = kd.nbmax + 2;
  int carry = 0;
  unsigned long long bsum = 0;
  if (lane == 0) seg[0] = 0;
  for (int base = 0; base < K; base += 64) {
    const int k = base + lane;
    int len = 0;
    if (k < K) {
      const int r = r0 + k;
      const int64_t b = c == 0 ? 0 : kd.split[(int64_t)r * per + c];
      const int64_t e = (c + 1 == ncell) ? kd.runs[r].nrec : kd.split[(int64_t)r * per + c + 1];
      sbase[k] = kd.runs[r].base + b * kTeraRecordBytes;
      len = (int)(e - b);
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
  if (lane == 0) *start_sum = (int64_t)bsum;
}

// 13 x 8-byte words per record, one wave per 64 consecutive output records. All 13 loads of a
// lane are issued before its first store: written as load -> store pairs, the compiler must assume
// the store may alias the next load and serializes 13 HBM round trips per 64 records. (Measured and
// dropped: non-temporal stores, and one whole record per lane as 16-byte pieces; both within noise,
// profiles/r3_kway_nt_ab.md, profiles/r3_kway_occupancy.md.)
__device__ __forceinline__ void kw_gather64(const uint8_t* const* sbase, const Elem* cur, int base, int valid,
                                            uint8_t* dst) {
  constexpr int kWords = kTeraRecordBytes / 8;
  // opaque per call: otherwise the per-word lane constants (record index, word offset) of all 13
  // words are hoisted out of the caller's loop and held in ~39 VGPRs, which caps the SIMD at 5 waves
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  unsigned long long src = 0;
  if (lane < valid) {
    const Elem e = cur[base + lane];
    const int run = (int)((e.lo >> 32) & 0xFFFF);
    src = (unsigned long long)(sbase[run] + (int64_t)(e.lo & 0xFFFFFFFFull) * kTeraRecordBytes);
  }
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
  uint64_t v[kWords];
  if (valid == 64) {  // straight-line: per-lane guards would split the stores into blocks that each drain vmcnt
#pragma unroll
    for (int j = 0; j < kWords; ++j) {
      const int w = j * 64 + lane;
      const int r = w / kWords;
      v[j] = ((const GlobalU64*)__shfl(src, r, 64))[w - r * kWords];
    }
#pragma unroll
    for (int j = 0; j < kWords; ++j) d[j * 64 + lane] = v[j];
    return;
  }
  const int words = valid * kWords;
#pragma unroll
  for (int j = 0; j < kWords; ++j) {
    const int w = j * 64 + lane;
    const int r = w / kWords;
    const unsigned long long s = __shfl(src, r < 64 ? r : 63, 64);
    v[j] = w < words ? ((const GlobalU64*)s)[w - r * kWords] : 0;
  }
#pragma unroll
  for (int j = 0; j < kWords; ++j) {
    const int w = j * 64 + lane;
    if (w < words) d[w] = v[j];
  }
}

// A cell that does not fit LDS (only massively duplicated keys): a wave-level priority queue. Lane l
// owns slices l, l + 64, ... (K <= 256: four per lane, their remaining and taken counts in registers);
// each step a wave argmin picks the next record. Wave 0 only.
__device__ void kw_overflow_pq(const KwayDesc& kd, const int* seg, const uint8_t* const* sbase, int K, int n,
                             uint8_t* obase) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  constexpr int kWords = kTeraRecordBytes / 8;
  constexpr int kPer = kKwMaxRuns / 64;
  int left[kPer], taken[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = lane + 64 * j;
    left[j] = k < K ? seg[k + 1] - seg[k] : 0;
    taken[j] = 0;
  }
  for (int64_t i = 0; i < n; ++i) {
    Elem best{~0ull, ~0ull};
    int bk = -1;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int k = lane + 64 * j;
      if (left[j] > 0) {
        const Elem e = load_key_elem(sbase[k] + (int64_t)taken[j] * kTeraRecordBytes, k, taken[j], kd.bad_layout);
        if (bk < 0 || kle(e, best)) {
          best = e;
          bk = k;
        }
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const uint64_t oh = __shfl_xor(best.hi, off, 64), ol = __shfl_xor(best.lo, off, 64);
      const int ok = __shfl_xor(bk, off, 64);
      const bool take = ok >= 0 && (bk < 0 || oh < best.hi || (oh == best.hi && ol < best.lo));
      if (take) {
        best.hi = oh;
        best.lo = ol;
        bk = ok;
      }
    }
    const int64_t pos = (int64_t)(best.lo & 0xFFFFFFFFull);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(sbase[bk] + pos * kTeraRecordBytes);
    uint64_t* dst = reinterpret_cast<uint64_t*>(obase + i * kTeraRecordBytes);
    if (lane < kWords) dst[lane] = src[lane];
    if (lane == (bk & 63)) {
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if ((bk >> 6) == j) {
          ++taken[j];
          --left[j];
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
  }
}

// F3: the K sorted slices of the cell's n keys at src[0, n) (slice k at [seg[k], seg[k+1])) merged pairwise
// in place, log2 K levels (merge path per thread over ceil(n / 256) outputs held in registers).
template <int ITEMS>
__device__ __forceinline__ void kw_merge_levels(Elem* src, const int* seg, int K, int n) {
  // outputs per thread: n spread evenly over the workgroup, so a cell filled to 65 % of its capacity
  // keeps every thread busy with a 65 % long merge chain
  const int ipt = (n + 256 - 1) / 256;
  const int o0 = threadIdx.x * ipt;
  uint64_t held_hi[ITEMS], held_lo[ITEMS];  // this thread's outputs of the current level
  for (int w = 1; w < K; w <<= 1) {
    if (o0 < n) {
      const int npairs = (K + 2 * w - 1) / (2 * w);
      // pair p covers segments [2pw, 2pw + 2w): find the pair holding output o0
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
      // merge path at diagonal o0 - a0 within the pair
      int d = o0 - a0, la = a1 - a0, lb = b1 - a1;
      int ml = d > lb ? d - lb : 0, mh = d < la ? d : la;
      while (ml < mh) {
        const int mid = (ml + mh) >> 1;
        if (kle(src[a0 + mid], src[a1 + d - 1 - mid]))
          ml = mid + 1;
        else
          mh = mid;
      }
      int ia = ml, ib = d - ml;
      const int todo = min(ipt, n - o0);
      // the two heads stay in registers: one LDS read per output (the side that advanced), clamped
      // to the cell so a run's end never reads past the buffer
      Elem va = src[min(a0 + ia, n - 1)], vb = src[min(a1 + ib, n - 1)];
#pragma unroll
      for (int k = 0; k < ITEMS; ++k) {
        if (k >= todo) continue;  // (not break: keeps the loop fully unrolled, held[] in registers)
        const int o = o0 + k;
        while (o == b1) {  // next pair (empty pairs are skipped)
          ++p;
          a0 = b1;
          a1 = seg[min((2 * p + 1) * w, K)];
          b1 = seg[min((2 * p + 2) * w, K)];
          la = a1 - a0;
          lb = b1 - a1;
          ia = 0;
          ib = 0;
          va = src[min(a0, n - 1)];
          vb = src[min(a1, n - 1)];
        }
        // straight-line step: bitwise conditions, the advancing side's next index selected, one
        // ds_read_b128 for the whole wave (as two exec-masked reads behind branches: same speed, more
        // LDS instructions; profiles/r4_kway_one_read_ab.md). Field-wise selects: a select of the two
        // structs becomes a scratch slot + indexed load.
        const bool take_a = (ib >= lb) | ((ia < la) & kle(va, vb));
        held_hi[k] = take_a ? va.hi : vb.hi;
        held_lo[k] = take_a ? va.lo : vb.lo;
        ia += take_a ? 1 : 0;
        ib += take_a ? 0 : 1;
        const Elem nv = src[min(take_a ? a0 + ia : a1 + ib, n - 1)];
        va.hi = take_a ? nv.hi : va.hi;
        va.lo = take_a ? nv.lo : va.lo;
        vb.hi = take_a ? vb.hi : nv.hi;
        vb.lo = take_a ? vb.lo : nv.lo;
      }
    }
    __syncthreads();
    // every thread has read the level: overwrite it with the merged order
    if (o0 < n) {
      const int todo = min(ipt, n - o0);
#pragma unroll
      for (int k = 0; k < ITEMS; ++k)
        if (k < todo) src[o0 + k] = Elem{held_hi[k], held_lo[k]};
    }
    __syncthreads();
  }
}

}  // namespace

// ITEMS records per thread: the cell capacity is ITEMS * 256 and the LDS buffer is dynamic, so
// smaller capacities fit more workgroups per CU. One cap x 16-byte buffer: a merge level keeps each
// thread's outputs in registers, waits for every thread to finish reading, then writes them back in
// place (two barriers per level), half the LDS of ping-pong buffers (+18.5 %, r3_kway_occupancy.md).
template <int ITEMS>
__global__ void __launch_bounds__(256) kway_tile_kernel(KwayDesc kd, uint8_t* out) {
  constexpr int kKwItems = ITEMS;
  constexpr int kKwThreads = 256;
  constexpr int kKwWaves = kKwThreads / 64;
  constexpr int kCap = ITEMS * kKwThreads;
  extern __shared__ __attribute__((aligned(16))) Elem kw_dyn[];
  Elem* bufA = kw_dyn;
  // per-slice tables behind the element buffer, sized by the plan's largest group (kd.kmax): a
  // 32-run round needs 388 bytes here, not the 2.5 KiB a static kKwMaxRuns table would pin
  const uint8_t** sbase = reinterpret_cast<const uint8_t**>(kw_dyn + kCap);  // slice starts
  int* seg = reinterpret_cast<int*>(sbase + kd.kmax);  // [K + 1] slice offsets within the cell
  __shared__ int64_t s_start;
  // The dispatcher deals workgroups round-robin over the 8 XCDs (each with its own L2); with the
  // swizzle, XCD x takes a contiguous block of cells, so neighbouring cells of a group (adjacent
  // slices of the same runs, sharing the boundary record lines) meet in one L2.
  int64_t b = blockIdx.x;
  {
    const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
    b = x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
  }
  // phase timestamps (tools only: kd.prof is null in production launches)
  auto stamp = [&](int k) {
    if (kd.prof && threadIdx.x == 0) kd.prof[b * 5 + k] = wall_clock64();
  };
  stamp(0);
  int lo = 0, hi = kd.G;  // cell_first[lo] <= b < cell_first[lo + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (kd.cell_first[mid] <= b)
      lo = mid;
    else
      hi = mid;
  }
  const int g = lo;
  const int c = (int)(b - kd.cell_first[g]);
  const int ncell = (int)(kd.cell_first[g + 1] - kd.cell_first[g]);
  const int r0 = kd.group_first[g], K = kd.group_first[g + 1] - r0;
  kw_slices(kd, c, ncell, r0, K, seg, sbase, &s_start);
  __syncthreads();
  stamp(1);
  const int n = seg[K];
  uint8_t* obase = out + (kd.group_out[g] + s_start) * kTeraRecordBytes;
  if (n > kCap) {  // uniform across the block
    if (threadIdx.x == 0) atomicAdd(kd.overflow, 1);
    kw_overflow_pq(kd, seg, sbase, K, n, obase);
    return;
  }
  // ---- F2: keys of every slice into LDS (all of a thread's key loads in flight at once)
  if (n > 0) {
    uint64_t w0[kKwItems], w1[kKwItems];
    int slv[kKwItems], posv[kKwItems];  // slice, record within the slice
#pragma unroll
    for (int k = 0; k < kKwItems; ++k) {
      // items past n re-read item n - 1: unguarded loads stay in one block and all stay in flight
      const int i = min(threadIdx.x + k * kKwThreads, n - 1);
      int sl = 0, sh = K;  // seg[sl] <= i < seg[sl + 1]
      while (sh - sl > 1) {
        const int mid = (sl + sh) >> 1;
        if (seg[mid] <= i)
          sl = mid;
        else
          sh = mid;
      }
      slv[k] = sl;
      posv[k] = i - seg[sl];
    }
#pragma unroll
    for (int k = 0; k < kKwItems; ++k) {
      const GlobalU64* rec = gptr(sbase[slv[k]] + (int64_t)posv[k] * kTeraRecordBytes);
      w0[k] = rec[0];
      w1[k] = rec[1];
    }
    int bad = 0;
#pragma unroll
    for (int k = 0; k < kKwItems; ++k) {
      const int i = threadIdx.x + k * kKwThreads;
      if (i < n) bufA[i] = key_elem(w0[k], w1[k], slv[k], posv[k], bad);  // ties: (slice, position) order
    }
    if (bad) *kd.bad_layout = 1;
  }
  __syncthreads();
  stamp(2);
  // ---- F3: pairwise merge levels inside LDS
  Elem* src = bufA;
  kw_merge_levels<kKwItems>(src, seg, K, n);
  stamp(3);
  // ---- F4: records in merged order straight to the output
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: a scalar loop
  for (int base = wave * 64; base < n; base += kKwWaves * 64) {
    const int valid = min(64, n - base);
    kw_gather64(sbase, src, base, valid, obase + (int64_t)base * kTeraRecordBytes);
  }
  if (kd.prof) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    stamp(4);
  }
}

// LDS-staged variant (KwayDesc::staged, UDA_KWAY_STAGED=1): every slice's records are copied into LDS
// once, as whole 16-byte chunks of the slice's aligned window (global_load_lds_dwordx4: per-lane global
// address, wave-linear LDS image), F2 reads the keys from there and F4 writes the output from there. In
// kway_tile_kernel F2 pulls each record's first line for its key and F4 pulls the whole record again
// after the merge, and in between the XCD's other cells have evicted it from L2: 2.07x the record bytes
// cross the fabric (profiles/r5_kway_roofline.md). Staged, each byte crosses once, at the price of a
// cap x 104-byte record image in LDS (cap 1024: 122 KB, one workgroup per CU; cap 512: two).
// LDS layout: keys[cap] | windows (cap*104 + kmax*32 + 1 KiB) | sbase[kmax] | seg[kmax+1] | wfirst[kmax+1] | roff[kmax]
template <int ITEMS>
__global__ void __launch_bounds__(256) kway_staged_kernel(KwayDesc kd, uint8_t* out) {
  constexpr int kCap = ITEMS * 256;
  constexpr int kWaves = 4;
  extern __shared__ __attribute__((aligned(16))) Elem kw_dyn[];
  Elem* keys = kw_dyn;
  uint8_t* win = reinterpret_cast<uint8_t*>(kw_dyn + kCap);
  const size_t win_bytes = (size_t)kCap * kTeraRecordBytes + (size_t)kd.kmax * 32 + 1024;
  const uint8_t** sbase = reinterpret_cast<const uint8_t**>(win + win_bytes);
  int* seg = reinterpret_cast<int*>(sbase + kd.kmax);
  int* wfirst = seg + kd.kmax + 1;  // [K + 1]: first 16-byte chunk of slice k's window
  int* roff = wfirst + kd.kmax + 1;  // [K]: offset of slice k's first record in its first chunk (0 or 8)
  __shared__ int64_t s_start;
  int64_t b = blockIdx.x;
  {
    const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8, slot = b / 8;
    b = x < r ? x * (q + 1) + slot : r * (q + 1) + (x - r) * q + slot;
  }
  int lo = 0, hi = kd.G;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (kd.cell_first[mid] <= b)
      lo = mid;
    else
      hi = mid;
  }
  const int g = lo;
  const int c = (int)(b - kd.cell_first[g]);
  const int ncell = (int)(kd.cell_first[g + 1] - kd.cell_first[g]);
  const int r0 = kd.group_first[g], K = kd.group_first[g + 1] - r0;
  kw_slices(kd, c, ncell, r0, K, seg, sbase, &s_start);
  __syncthreads();
  const int n = seg[K];
  uint8_t* obase = out + (kd.group_out[g] + s_start) * kTeraRecordBytes;
  if (n > kCap) {
    if (threadIdx.x == 0) atomicAdd(kd.overflow, 1);
    kw_overflow_pq(kd, seg, sbase, K, n, obase);
    return;
  }
  if (n == 0) return;
  // ---- windows: slice k's bytes rounded out to 16-byte chunks, the windows back to back (wave 0 scans)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int carry = 0;
    if (lane == 0) wfirst[0] = 0;
    for (int base = 0; base < K; base += 64) {
      const int k = base + lane;
      int chunks = 0;
      if (k < K) {
        const int len = seg[k + 1] - seg[k];
        const uintptr_t a = (uintptr_t)sbase[k];
        roff[k] = (int)(a & 15);
        if (len > 0) chunks = (int)((((a + (uintptr_t)len * kTeraRecordBytes + 15) & ~(uintptr_t)15) - (a & ~(uintptr_t)15)) >> 4);
      }
      int x = chunks;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (k < K) wfirst[k + 1] = carry + x;
      carry += __shfl(x, 63, 64);
    }
  }
  __syncthreads();
  // ---- stage: chunk i of the flattened windows lands at win + 16 i. A window's last chunk may run 8 bytes
  // past the slice's last record, possibly past its allocation: that lane reads a chunk inside the slice
  // instead and the chunk's 8 valid bytes are patched below.
  const int T = wfirst[K];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform
  for (int base = wave * 64; base < T; base += kWaves * 64) {
    const int i = base + lane;
    const int ic = min(i, T - 1);
    int sl = 0, sh = K;  // wfirst[sl] <= ic < wfirst[sl + 1]
    while (sh - sl > 1) {
      const int mid = (sl + sh) >> 1;
      if (wfirst[mid] <= ic)
        sl = mid;
      else
        sh = mid;
    }
    const uintptr_t a0 = (uintptr_t)sbase[sl] & ~(uintptr_t)15;
    const uintptr_t end = (uintptr_t)sbase[sl] + (uintptr_t)(seg[sl + 1] - seg[sl]) * kTeraRecordBytes;
    uintptr_t src = a0 + (uintptr_t)(ic - wfirst[sl]) * 16;
    if (src + 16 > end) src = a0;  // the tail chunk (patched below), or a lane past T
    // C casts: the address-space conversions have no named-cast form
    __builtin_amdgcn_global_load_lds((const GlobalVoid*)src, (LdsVoid*)(win + (size_t)base * 16), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256) {
    const int len = seg[k + 1] - seg[k];
    const uintptr_t end = (uintptr_t)sbase[k] + (uintptr_t)len * kTeraRecordBytes;
    if (len > 0 && (end & 15))
      *reinterpret_cast<uint64_t*>(win + (size_t)(wfirst[k + 1] - 1) * 16) = *reinterpret_cast<const GlobalU64*>(end - 8);
  }
  __syncthreads();
  auto rec = [&](int sl, int pos) {
    return win + (size_t)wfirst[sl] * 16 + roff[sl] + (size_t)pos * kTeraRecordBytes;
  };
  // ---- F2 from LDS
  {
    int bad = 0;
    for (int i = threadIdx.x; i < n; i += 256) {
      int sl = 0, sh = K;
      while (sh - sl > 1) {
        const int mid = (sl + sh) >> 1;
        if (seg[mid] <= i)
          sl = mid;
        else
          sh = mid;
      }
      const uint64_t* w = reinterpret_cast<const uint64_t*>(rec(sl, i - seg[sl]));
      keys[i] = key_elem(w[0], w[1], sl, i - seg[sl], bad);
    }
    if (bad) *kd.bad_layout = 1;
  }
  __syncthreads();
  // ---- F3
  kw_merge_levels<ITEMS>(keys, seg, K, n);
  // ---- F4 from LDS: one wave per 64 output records, 13 consecutive 8-byte words per record
  constexpr int kWords = kTeraRecordBytes / 8;
  for (int base = wave * 64; base < n; base += kWaves * 64) {
    const int valid = min(64, n - base);
    uint32_t my = 0;  // LDS offset of this lane's record
    if (lane < valid) {
      const Elem e = keys[base + lane];
      my = (uint32_t)(rec((int)((e.lo >> 32) & 0xFFFF), (int)(e.lo & 0xFFFFFFFFull)) - win);
    }
    uint64_t* d = reinterpret_cast<uint64_t*>(obase + (int64_t)base * kTeraRecordBytes);
    const int words = valid * kWords;
#pragma unroll
    for (int j = 0; j < kWords; ++j) {
      const int w = j * 64 + lane;
      const int r = w / kWords;
      const uint32_t o = __shfl(my, r < 64 ? r : 63, 64);
      if (w < words) d[w] = *reinterpret_cast<const uint64_t*>(win + o + (uint32_t)(w - r * kWords) * 8);
    }
  }
}

void launch_pick_splitters(const Elem* samples, const int64_t* gsamp_off, const int64_t* gcells, int G, int nbmax,
                           Elem* bounds, hipStream_t s) {
  const int64_t n = (int64_t)G * nbmax;
  if (n <= 0) return;
  hipLaunchKernelGGL(pick_splitters_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, samples, gsamp_off,
                     gcells, G, nbmax, bounds);
}

void launch_split_sampled(uint8_t* const* bases, const int64_t* nrec, const Elem* samples, const int64_t* soff,
                          int64_t every, const Elem* bounds, const int* run_bound_set, int nruns, int nb, int64_t* out,
                          hipStream_t s) {
  const int64_t total = (int64_t)nruns * (nb + 2);
  if (total <= 0) return;
  hipLaunchKernelGGL(split_sampled_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, bases, nrec,
                     samples, soff, every, bounds, run_bound_set, nruns, nb, out);
}

int kway_cap_supported(int cap) { return cap == 2048 || cap == 1792 || cap == 1536 || cap == 1024 || cap == 512; }

namespace {
template <int ITEMS>
void launch_kway(const KwayDesc& kd, int64_t ncells, uint8_t* out, hipStream_t s) {
  const size_t elems = sizeof(Elem) * (size_t)(ITEMS * 256);
  auto tables = [](int k) { return (size_t)k * sizeof(void*) + (size_t)(k + 1) * sizeof(int); };
  if (kd.kmax < 1 || kd.kmax > kKwMaxRuns) throw std::runtime_error("kway: bad runs per group " + std::to_string(kd.kmax));
  const size_t lds = (elems + tables(kd.kmax) + 15) & ~(size_t)15;
  static std::once_flag once;
  static hipError_t attr = hipSuccess;
  std::call_once(once, [elems, tables] {  // dynamic LDS above the 64 KiB default (gfx950 has 160 KiB per CU)
    attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kway_tile_kernel<ITEMS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)(elems + tables(kKwMaxRuns) + 16));
    // some runtimes refuse the attribute for template kernels: harmless while a launch stays within the
    // default, and the error must not linger for the next hipGetLastError
    if (attr != hipSuccess) (void)hipGetLastError();
  });
  if (attr != hipSuccess && lds > (64u << 10))
    throw std::runtime_error(std::string("kway: cannot raise the LDS limit: ") + hipGetErrorString(attr));
  hipLaunchKernelGGL((kway_tile_kernel<ITEMS>), dim3((unsigned)ncells), dim3(256), lds, s, kd, out);
}
}  // namespace

template <int ITEMS>
void launch_kway_staged(const KwayDesc& kd, int64_t ncells, uint8_t* out, hipStream_t s) {
  auto lds_for = [](int k) {
    const size_t cap = (size_t)ITEMS * 256;
    return cap * sizeof(Elem) + cap * kTeraRecordBytes + (size_t)k * 32 + 1024 + (size_t)k * sizeof(void*) +
           (size_t)(3 * k + 2) * sizeof(int) + 16;
  };
  if (kd.kmax < 1 || kd.kmax > kKwMaxRuns) throw std::runtime_error("kway: bad runs per group " + std::to_string(kd.kmax));
  const size_t lds = lds_for(kd.kmax);
  if (lds > (160u << 10)) throw std::runtime_error("kway staged: cell of " + std::to_string(ITEMS * 256) + " records with " +
                                                   std::to_string(kd.kmax) + " runs needs " + std::to_string(lds) +
                                                   " bytes of LDS");
  static std::once_flag once;
  static hipError_t attr = hipSuccess;
  std::call_once(once, [lds_for] {
    attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kway_staged_kernel<ITEMS>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_for(kKwMaxRuns));
    if (attr != hipSuccess) (void)hipGetLastError();
  });
  if (attr != hipSuccess && lds > (64u << 10))
    throw std::runtime_error(std::string("kway staged: cannot raise the LDS limit: ") + hipGetErrorString(attr));
  hipLaunchKernelGGL((kway_staged_kernel<ITEMS>), dim3((unsigned)ncells), dim3(256), lds, s, kd, out);
}

void launch_kway_tiles(const KwayDesc& kd, int64_t ncells, uint8_t* out, hipStream_t s) {
  if (ncells <= 0) return;
  if (kd.staged) {
    switch (kd.cap) {
      case 1024: launch_kway_staged<4>(kd, ncells, out, s); return;
      case 512: launch_kway_staged<2>(kd, ncells, out, s); return;
      default: throw std::runtime_error("kway staged: cell capacity must be 512 or 1024 (UDA_KWAY_CAP)");
    }
  }
  switch (kd.cap) {
    case 2048: launch_kway<8>(kd, ncells, out, s); break;
    case 1792: launch_kway<7>(kd, ncells, out, s); break;  // 28.4 KiB, 5 workgroups per CU
    case 1536: launch_kway<6>(kd, ncells, out, s); break;
    case 1024: launch_kway<4>(kd, ncells, out, s); break;
    case 512: launch_kway<2>(kd, ncells, out, s); break;
    default: throw std::runtime_error("kway: unsupported cell capacity " + std::to_string(kd.cap));
  }
}

}  // namespace gpu
}  // namespace uda
