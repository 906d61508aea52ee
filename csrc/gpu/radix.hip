// F8: map-side sort of TeraSort records on the device (gfx950, wave64) — an LSD radix sort on the
// 10-byte key followed by one record gather.
//
// Reference context: UDA only shuffles; each Hadoop map task sorts its spill with a CPU quicksort
// before writing the IFile partitions the reducers fetch ("a full sort, not
// only a merge, if runs arrive unsorted"). Here the map output is generated unsorted in HBM and sorted
// in place, so the reduce side sees runs produced by an actual sort.
//
// Layout: a 16-byte SortKey {hi = key bytes 0..7, lo = key bytes 8..9, idx = record ordinal} per
// record. Ten stable 8-bit passes (two over lo, eight over hi) each run
//   hist    : one workgroup per 4096-key tile, LDS histogram of the pass digit, wave-aggregated
//             (the lanes of a wave holding the same digit add once);
//   scan    : one workgroup per digit scans that digit's per-tile counts (digit-major table);
//   scatter : each tile re-reads its keys in 16 striped rounds of 256 (so (round, wave, lane) order is
//             input order) and ranks them inside the wave by an 8-bit ballot match: a lane's peers are
//             the lanes whose digit equals its own, its rank the peers below it. Per-wave digit counts
//             go through LDS so a key's slot = digit base + tile offset + earlier rounds + earlier
//             waves + rank: stable, which LSD needs. The whole 4096-key tile is staged in LDS (64 KiB)
//             in digit order before any store, so a digit's ~16 keys leave as one 256-byte run of
//             addresses (staging one 256-key round at a time left ~1 key per digit per store and
//             wrote 1.76x the key bytes to HBM: profiles/r2_radix_pmc.md).
// Then a gather moves each 104-byte record once (13 lanes per record, 8-byte words).
#include "kernels.h"

namespace uda {
namespace gpu {

namespace {

struct alignas(16) SortKey {
  uint64_t hi;   // key bytes 0..7, big-endian order
  uint32_t lo;   // key bytes 8..9
  uint32_t idx;  // record ordinal in the run
};

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;
constexpr int kBins = 256;
constexpr int kPasses = 10;
constexpr int kWords = kTeraRecordBytes / 8;  // 13

__device__ __forceinline__ uint32_t digit_of(const SortKey& k, int pass) {
  return pass < 2 ? (k.lo >> (8 * pass)) & 0xFF : (uint32_t)(k.hi >> (8 * (pass - 2))) & 0xFF;
}

// Lanes of this wave whose digit equals this lane's (8 ballots over the digit bits).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1;
    const uint64_t m = __ballot(bit);
    peers &= bit ? m : ~m;
  }
  return peers;
}

__device__ __forceinline__ uint64_t lanes_below() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Block-wide exclusive scan of one value per thread (256 threads); returns the thread's prefix and
// writes the block total to *total. Uses `tmp` (kWaves entries of LDS).
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* tmp, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const uint32_t t = tmp[w];
    if (w < wave) before += t;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

__device__ __forceinline__ void load_key(const uint8_t* rec, uint64_t* hi, uint32_t* lo) {
  // [0x0B][0x5B][0x0A][k0..k9]...: key bytes 0..4 are record bytes 3..7, 5..9 are bytes 8..12
  const uint64_t w0 = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(rec));
  const uint64_t w1 = __builtin_bswap64(*reinterpret_cast<const uint64_t*>(rec + 8));
  *hi = (w0 << 24) | (w1 >> 40);
  *lo = (uint32_t)((w1 >> 24) & 0xFFFF);
}

__global__ void __launch_bounds__(kThreads) rs_extract_kernel(const uint8_t* base, int64_t n, SortKey* out) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  SortKey k;
  load_key(base + i * kTeraRecordBytes, &k.hi, &k.lo);
  k.idx = (uint32_t)i;
  out[i] = k;
}

__global__ void __launch_bounds__(kThreads) rs_hist_kernel(const SortKey* __restrict__ in, int64_t n, int pass,
                                                           uint32_t* __restrict__ hist, int ntiles) {
  __shared__ uint32_t h[kBins];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll 4
  for (int k = 0; k < kItems; ++k) {
    const int64_t i = base + k * kThreads + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? digit_of(in[i], pass) : 0;
    const uint64_t peers = match_digit(d, valid);
    if (valid && (peers & lanes_below()) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
  }
  __syncthreads();
  hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// One workgroup per digit: exclusive scan of the digit's per-tile counts in place; totals[d] = sum.
__global__ void __launch_bounds__(kThreads) rs_scan_kernel(uint32_t* __restrict__ hist, int ntiles,
                                                           uint32_t* __restrict__ totals) {
  __shared__ uint32_t tmp[kWaves];
  uint32_t* row = hist + (size_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (int c = 0; c < ntiles; c += kThreads * 4) {
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = c + threadIdx.x * 4 + j;
      v[j] = t < ntiles ? row[t] : 0;
      s += v[j];
    }
    uint32_t total;
    uint32_t pre = block_exclusive_scan(s, tmp, &total) + carry;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = c + threadIdx.x * 4 + j;
      if (t < ntiles) row[t] = pre;
      pre += v[j];
    }
    carry += total;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

__global__ void __launch_bounds__(kThreads) rs_scatter_kernel(const SortKey* __restrict__ in, SortKey* __restrict__ out,
                                                              int64_t n, int pass, const uint32_t* __restrict__ hist,
                                                              const uint32_t* __restrict__ totals, int ntiles) {
  __shared__ uint32_t gbase[kBins];         // global slot of the tile's first key of each digit
  __shared__ uint32_t tstart[kBins];        // the digit's first slot in the tile's LDS staging
  __shared__ uint32_t run[kBins];           // keys of the digit staged by earlier rounds
  __shared__ uint32_t wcnt[kWaves][kBins];  // per-wave digit counts -> exclusive prefixes
  __shared__ SortKey stage[kTile];          // the whole tile in digit order
  __shared__ uint32_t tmp[kWaves];
  const int t = threadIdx.x, wave = t >> 6;
  const int b = blockIdx.x;
  {
    // the scan left hist[d][b] = keys of digit d in tiles before b; the tile's own count is the
    // difference to the next tile (or to the digit total)
    const uint32_t h = hist[(size_t)t * ntiles + b];
    const uint32_t cnt = (b + 1 < ntiles ? hist[(size_t)t * ntiles + b + 1] : totals[t]) - h;
    uint32_t all;
    const uint32_t digit_off = block_exclusive_scan(totals[t], tmp, &all);
    gbase[t] = digit_off + h;
    tstart[t] = block_exclusive_scan(cnt, tmp, &all);
    run[t] = 0;
  }
  const int64_t base = (int64_t)b * kTile;
  for (int k = 0; k < kItems; ++k) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) wcnt[w][t] = 0;
    __syncthreads();
    const int64_t i = base + k * kThreads + t;
    const bool valid = i < n;
    SortKey key{};
    if (valid) key = in[i];
    const uint32_t d = valid ? digit_of(key, pass) : 0;
    const uint64_t peers = match_digit(d, valid);
    const uint32_t rank = (uint32_t)__popcll(peers & lanes_below());
    if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    // thread t owns digit t: exclusive prefix over the waves and the round's count
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const uint32_t c = wcnt[w][t];
      wcnt[w][t] = s;
      s += c;
    }
    __syncthreads();
    // (round, wave, lane) order is input order: the slot keeps the sort stable
    if (valid) stage[tstart[d] + run[d] + wcnt[wave][d] + rank] = key;
    __syncthreads();
    run[t] += s;
  }
  __syncthreads();
  // the tile's keys leave in digit order: a digit's keys (16 on average) are one run of addresses
  const int nt = (int)min<int64_t>(kTile, n - base);
  for (int x = t; x < nt; x += kThreads) {
    const SortKey k2 = stage[x];
    const uint32_t d2 = digit_of(k2, pass);
    out[(size_t)gbase[d2] + (uint32_t)x - tstart[d2]] = k2;
  }
}

__global__ void __launch_bounds__(kThreads) rs_gather_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                             const SortKey* __restrict__ keys, int64_t n, int eof) {
  const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t i = g / kWords;
  if (i >= n) return;
  const int w = (int)(g - i * kWords);
  dst[i * kWords + w] = src[(int64_t)keys[i].idx * kWords + w];
  if (eof && g == 0) {  // IFile EOF marker VInt(-1) VInt(-1) after the last record
    uint8_t* e = reinterpret_cast<uint8_t*>(dst + n * kWords);
    e[0] = 0xFF;
    e[1] = 0xFF;
  }
}

int64_t tiles_of(int64_t n) { return (n + kTile - 1) / kTile; }

}  // namespace

int64_t sort_fixed_ws_bytes(int64_t n) {
  const int64_t keys = ((n * (int64_t)sizeof(SortKey) + 255) & ~255ll) * 2;
  const int64_t hist = ((tiles_of(n) * kBins * 4 + 255) & ~255ll) + 1024;
  const int64_t recs = (n * kTeraRecordBytes + 255) & ~255ll;
  return keys + hist + recs;
}

uint8_t* sort_fixed_ws_records(void* ws, int64_t n) {
  const int64_t kb = (n * (int64_t)sizeof(SortKey) + 255) & ~255ll;
  return static_cast<uint8_t*>(ws) + 2 * kb + ((tiles_of(n) * kBins * 4 + 255) & ~255ll) + 1024;
}

void launch_sort_fixed_run(uint8_t* base, int64_t n, void* ws, hipStream_t s, bool staged) {
  if (n <= 0) return;
  if (n == 1 && !staged) return;
  uint8_t* p = static_cast<uint8_t*>(ws);
  const int64_t kb = (n * (int64_t)sizeof(SortKey) + 255) & ~255ll;
  SortKey* a = reinterpret_cast<SortKey*>(p);
  SortKey* b = reinterpret_cast<SortKey*>(p + kb);
  const int64_t ntiles = tiles_of(n);
  uint32_t* hist = reinterpret_cast<uint32_t*>(p + 2 * kb);
  uint32_t* totals = reinterpret_cast<uint32_t*>(p + 2 * kb + ((ntiles * kBins * 4 + 255) & ~255ll));
  uint8_t* recs = sort_fixed_ws_records(ws, n);
  // staged: the unsorted records are in the workspace's record area and the sort gathers them into
  // `base` (plus the EOF marker); otherwise they are at `base` and are copied aside first
  const uint8_t* src = staged ? recs : base;
  hipLaunchKernelGGL(rs_extract_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, s, src, n, a);
  for (int pass = 0; pass < kPasses; ++pass) {
    hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)ntiles), dim3(kThreads), 0, s, a, n, pass, hist, (int)ntiles);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(kBins), dim3(kThreads), 0, s, hist, (int)ntiles, totals);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3((unsigned)ntiles), dim3(kThreads), 0, s, a, b, n, pass, hist, totals,
                       (int)ntiles);
    SortKey* t = a;
    a = b;
    b = t;
  }
  // kPasses is even: the sorted keys are back in the first buffer
  if (!staged) (void)hipMemcpyAsync(recs, base, (size_t)(n * kTeraRecordBytes), hipMemcpyDeviceToDevice, s);
  const int64_t words = n * kWords;
  hipLaunchKernelGGL(rs_gather_kernel, dim3((unsigned)((words + kThreads - 1) / kThreads)), dim3(kThreads), 0, s,
                     reinterpret_cast<const uint64_t*>(recs), reinterpret_cast<uint64_t*>(base), a, n, staged ? 1 : 0);
}

}  // namespace gpu
}  // namespace uda
