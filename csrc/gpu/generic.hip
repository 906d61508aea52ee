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
#include <cstdlib>
#include "kernels.h"
#include "uda/compare.h"
#include "uda/vint.h"

namespace uda {
namespace gpu {

namespace {

// F1 in two passes.
//  pass 1 (one wave per run, serial along the run): the run streams through LDS in 4 KiB chunks
//    (the next chunk is fetched into registers while the current one is walked); lane 0 follows
//    the record chain decoding the two VInt headers from LDS and leaves a checkpoint per chunk:
//    the offset of the first record starting in the chunk and the number of records starting in it.
//  pass 2 (one wave per chunk, all chunks of all runs in parallel): each chunk is staged in LDS
//    again and re-walked from its checkpoint, writing the record offsets.
constexpr int kF1Chunk = 4096;
constexpr int kF1Halo = 32;
constexpr int kF1Lanes = 64;
constexpr int kF1Bytes = kF1Chunk / kF1Lanes;  // 64 bytes per lane

template <class BP>
__device__ __forceinline__ int lds_vint(BP b, int p, int lim, int64_t* v) {
  if (p >= lim) return 0;
  const int8_t f = (int8_t)b[p];
  if (f >= -112) {
    *v = f;
    return 1;
  }
  const bool neg = f < -120;
  const int n = neg ? (-120 - f) : (-112 - f);
  if (p + 1 + n > lim) return 0;
  int64_t t = 0;
  for (int i = 0; i < n; ++i) t = (t << 8) | b[p + 1 + i];
  if (neg) t ^= -1ll;
  *v = t;
  return n + 1;
}

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;  // unaligned 16-byte access (legal for global memory)

// Load bytes [at, at+64) of a run (zero beyond n) into registers. Runs start at any byte, so the
// full-width case uses unaligned 16-byte loads (a byte-at-a-time fallback costs 64 loads per lane).
__device__ __forceinline__ void f1_fetch64(const uint8_t* p, int64_t n, int64_t at, uint32_t (&w)[16]) {
  if (at + 64 <= n) {
    const u32x4_u* q = reinterpret_cast<const u32x4_u*>(p + at);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 v = q[k];
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      uint32_t x = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t i = at + 4 * k + b;
        x |= (uint32_t)(i < n ? p[i] : 0) << (8 * b);
      }
      w[k] = x;
    }
  }
}

__device__ __forceinline__ void f1_stage(uint8_t* buf, int lane, const uint32_t (&w)[16]) {
  uint32_t* d = reinterpret_cast<uint32_t*>(buf + lane * kF1Bytes);
#pragma unroll
  for (int k = 0; k < 16; ++k) d[k] = w[k];
}

// Decode the record at LDS position i; returns its size, 0 for EOF, -1 for corrupt/truncated.
// Fast path: both VInt headers are single bytes (lengths < 128, the common case); the two header
// bytes come from two independent aligned dword reads instead of two dependent byte reads.
// partial: the run is a landed prefix of a stream still arriving; a record cut by its end (header or
// body) ends it like the EOF marker (0), so rec_bytes is the prefix's last complete record end.
__device__ __forceinline__ int64_t f1_record(const uint8_t* buf, int i, int lim, int64_t remain, bool partial) {
  if (i + 2 <= lim) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(buf + (i & ~3));
    const uint64_t two = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    const int sh = (i & 3) * 8;
    const int8_t b0 = (int8_t)(two >> sh), b1 = (int8_t)(two >> (sh + 8));
    if (b0 >= 0 && b1 >= 0) {
      const int64_t sz = 2 + (int64_t)b0 + (int64_t)b1;
      return sz > remain ? (partial ? 0 : -1) : sz;
    }
  }
  int64_t kl = 0, vl = 0;
  const int a = lds_vint(buf, i, lim, &kl);
  const int b = a ? lds_vint(buf, i + a, lim, &vl) : 0;
  if (a == 0 || b == 0) return partial && remain < 20 ? 0 : -1;  // header cut by the prefix end
  if (kl == -1 && vl == -1) return 0;
  if (kl < 0 || vl < 0) return -1;
  const int64_t sz = a + b + kl + vl;
  return sz > remain ? (partial ? 0 : -1) : sz;
}

// The general decoder alone (multi-byte VInt headers, the EOF marker, a record at the run's tail):
// reads only bytes below lim.
template <class BP>
__device__ __forceinline__ int64_t f1_record_slow(BP buf, int i, int lim, int64_t remain, bool partial) {
  int64_t kl = 0, vl = 0;
  const int a = lds_vint(buf, i, lim, &kl);
  const int b = a ? lds_vint(buf, i + a, lim, &vl) : 0;
  if (a == 0 || b == 0) return partial && remain < 20 ? 0 : -1;
  if (kl == -1 && vl == -1) return 0;
  if (kl < 0 || vl < 0) return -1;
  const int64_t sz = a + b + kl + vl;
  return sz > remain ? (partial ? 0 : -1) : sz;
}

typedef __attribute__((address_space(1))) const uint8_t GlobalU8;

template <bool kProf>
__global__ void __launch_bounds__(kF1Lanes) f1_scan_kernel(uint8_t* const* bases, const int64_t* nbytes,
                                                           const int64_t* chunk_base, int64_t* ck_start,
                                                           int64_t* ck_count, int64_t* counts, int64_t* rec_bytes,
                                                           int* status, uint64_t* prof, const int* run_ids,
                                                           int partial) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kF1Chunk + 64];
  const int r = run_ids ? run_ids[blockIdx.x] : (int)blockIdx.x;
  const int lane = threadIdx.x;
  const uint8_t* p = bases[r];
  const int64_t n = nbytes[r];
  const int64_t cb = chunk_base[r];
  uint32_t cur[16], nxt[16];
  f1_fetch64(p, n, (int64_t)lane * kF1Bytes, cur);
  int64_t pos = 0, cnt = 0;
  int st = 0;
  bool done = false;
  uint64_t t_stage = 0, t_walk = 0, t0 = 0;
  int64_t c = 0;
  for (int64_t c0 = 0; c0 < n && !done; c0 += kF1Chunk, ++c) {
    if (kProf) t0 = stamp();
    f1_fetch64(p, n, c0 + kF1Chunk + (int64_t)lane * kF1Bytes, nxt);  // prefetch
    f1_stage(buf, lane, cur);
    if (lane == 0) {  // halo: the first bytes of the next chunk
      uint32_t* h = reinterpret_cast<uint32_t*>(buf + kF1Chunk);
#pragma unroll
      for (int k = 0; k < kF1Halo / 4; ++k) h[k] = nxt[k];
    }
    __syncthreads();
    if (kProf) {
      const uint64_t t1 = stamp();
      t_stage += t1 - t0;
      t0 = t1;
    }
    if (lane == 0) {
      const int lim = (int)((n - c0) < (int64_t)(kF1Chunk + kF1Halo) ? (n - c0) : (kF1Chunk + kF1Halo));
      const int64_t end = c0 + (lim < kF1Chunk ? lim : kF1Chunk);
      int64_t here = 0;
      ck_start[cb + c] = pos;  // first record at or after c0 (or the end)
      while (pos < end) {
        const int64_t sz = f1_record(buf, (int)(pos - c0), lim, n - pos, partial != 0);
        if (sz <= 0) {
          if (sz < 0) st = 1;
          done = true;
          break;
        }
        pos += sz;
        ++here;
      }
      ck_count[cb + c] = here;
      cnt += here;
    }
    done = __shfl(done ? 1 : 0, 0, 64) != 0;
    if (kProf) t_walk += stamp() - t0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) cur[k] = nxt[k];
  }
  if (lane == 0) {
    // chunks after an early EOF carry no records
    const int64_t nchunks = (n + kF1Chunk - 1) / kF1Chunk;
    for (int64_t k = c; k < nchunks; ++k) {
      ck_start[cb + k] = pos;
      ck_count[cb + k] = 0;
    }
    counts[r] = cnt;
    rec_bytes[r] = pos;
    status[r] = st;
    if (kProf) {
      prof[2 * r] = t_stage;
      prof[2 * r + 1] = t_walk;
    }
  }
}

// ---- F1 pass 1, parallel form (chunk transfer functions).
// The record chain of a run is a composition of per-chunk functions: entering chunk c at offset e
// (the first record start at or after the chunk's first byte, e < kF1Entries when records are at
// most kF1Entries bytes), the chain leaves the chunk at a known offset after a known number of
// records. (1) f1_fn: one wave per chunk tabulates that function for all kF1Entries entries (4
// chains per lane walked in lockstep over the LDS-staged chunk). (2) f1_super: one wave per
// superchunk of kF1Super chunks composes the chunk functions for every entry. (3) f1_top: one lane
// per run composes superchunks from offset 0 (the only serial step: run_bytes / 256 KiB hops).
// (4) f1_expand: one lane per superchunk replays its true entry through its chunks, emitting the
// same per-chunk checkpoints as the serial scan. A run whose true chain needs an entry beyond the
// table (a record longer than kF1Entries bytes straddles a chunk) is reported with status 2 and
// re-indexed by the serial scan.
constexpr int kF1Entries = 256;
constexpr int kF1Super = 64;
constexpr int kF1FnWaves = 4;
constexpr int kF1Warm = 2;  // lockstep steps of all chains before the survivors are compacted
constexpr int kF1Chase = 8;  // survivors per chunk handed to f1_chase_kernel (more: walked in f1_fn)
constexpr int32_t kFnInvalid = INT32_MIN;      // corrupt/truncated record on this chain
constexpr int32_t kFnFallback = INT32_MIN + 1;  // exit offset not representable
constexpr int64_t kSupInvalid = -1, kSupFallback = -2;  // super codes; EOF at q -> -3 - q

// One step of an F1 chain inside chunk-relative bytes buf[0, lim): decode the record at pos (two
// sign-extending byte reads and a few 32-bit ops in the common case; multi-byte VInt headers go to
// the general decoder). Key framing check (lengths < 128): a Text key starts with its own VInt
// length (klen - 1), a BytesWritable key with a 4-byte big-endian klen - 4. A chain entered at a
// byte that is not a record start almost never passes, so garbage chains end after one step; a
// failing chain ends as "fallback", never "corrupt": if it were the true chain, the run is
// re-indexed by the serial scan, which does not apply the check. kGuard: reads at or past lim
// return 0 (global memory, where bytes past the run are not ours; the LDS stage is zero-padded).
template <bool kGuard, class BP>
__device__ __forceinline__ void f1_step(BP buf, int lim, int64_t nrel64, int nrel, int end_rel, int key_kind, int& pos,
                                        int& cnt, int& code, bool& alive, bool partial) {
  auto rd = [&](int i) -> int { return kGuard && i >= lim ? 0 : (int)(int8_t)buf[i]; };
  const int p = alive ? pos : 0;
  const int b0 = rd(p), b1 = rd(p + 1);
  int sz = 2 + b0 + b1;
  bool fallback = false;
  if (alive && ((b0 | b1) < 0 || p + 2 > lim)) {
    const int64_t s64 = f1_record_slow(buf, p, lim, nrel64 - p, partial);
    fallback = s64 > (int64_t)(1 << 30);
    sz = fallback ? 1 : (int)s64;
  } else if (p + sz > nrel) {
    sz = partial && p + sz > nrel64 ? 0 : -1;  // partial: cut by the landed prefix's end
  }
  if (key_kind == (int)KeyKind::kText && (b0 | b1) >= 0 && p + 3 <= lim)
    fallback = fallback || !(b0 >= 1 && rd(p + 2) == b0 - 1);
  else if (key_kind == (int)KeyKind::kBytes && (b0 | b1) >= 0 && p + 6 <= lim)
    fallback = fallback || !(b0 >= 4 && rd(p + 2) == 0 && rd(p + 3) == 0 && rd(p + 4) == 0 && (rd(p + 5) & 0xFF) == b0 - 4);
  const bool bad = sz <= 0;
  const int np = p + sz;
  const bool fin = !bad && (np >= end_rel || fallback);
  if (alive) {
    code = bad ? (sz == 0 ? -1 - p : kFnInvalid) : fallback ? kFnFallback : fin ? np : code;
    pos = bad ? pos : np;
    cnt += bad ? 0 : 1;
  }
  alive = alive && !(bad || fin);
}

__global__ void __launch_bounds__(64 * kF1FnWaves) f1_fn_kernel(uint8_t* const* bases, const int64_t* nbytes,
                                                                 const int64_t* chunk_base, const int32_t* chunk_run,
                                                                 int64_t nchunks, int32_t* fx, int32_t* fn,
                                                                 int key_kind, int32_t* chase, int32_t* chase_n,
                                                                 int partial) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kF1FnWaves][kF1Chunk + 64];
  __shared__ int f1_live[kF1FnWaves][3 * kF1Entries];  // surviving chains: entry, position, count
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wv: wave-uniform
  const int64_t c = (int64_t)blockIdx.x * kF1FnWaves + wv;
  const bool valid = c < nchunks;
  uint8_t* buf = lds[wv];
  int r = 0;
  int64_t n = 0, c0 = 0;
  if (valid) {
    r = chunk_run[c];
    n = nbytes[r];
    c0 = (c - chunk_base[r]) * kF1Chunk;
    const uint8_t* p = bases[r];
    uint32_t w[16];
    f1_fetch64(p, n, c0 + (int64_t)lane * kF1Bytes, w);
    f1_stage(buf, lane, w);
    if (lane == 0) {
      uint32_t h[16];
      f1_fetch64(p, n, c0 + kF1Chunk, h);
      uint32_t* d = reinterpret_cast<uint32_t*>(buf + kF1Chunk);
#pragma unroll
      for (int k = 0; k < 16; ++k) d[k] = h[k];
    }
  }
  __syncthreads();
  if (!valid) return;
  const int end_rel = (int)min((int64_t)kF1Chunk, n - c0);
  const int lim = (int)min(n - c0, (int64_t)(kF1Chunk + kF1Halo));
  const int64_t nrel64 = n - c0;
  const int nrel = (int)min(nrel64, (int64_t)(1 << 30));  // records must end by here (fast path)
  auto step = [&](int& pos, int& cnt, int& code, bool& alive) {
    f1_step<false>(buf, lim, nrel64, nrel, end_rel, key_kind, pos, cnt, code, alive, partial != 0);
  };
  int32_t* x = fx + c * kF1Entries;
  int32_t* m = fn + c * kF1Entries;
  // Phase 1: all kF1Entries chains (4 per lane) for a few lockstep steps. Chains from offsets that
  // are not record starts decode garbage lengths and die within ~2-3 steps; only the true chain and
  // the few that fall onto it survive.
  int pos[4], cnt[4], code[4];
  bool alive[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pos[j] = lane + 64 * j;
    cnt[j] = 0;
    code[j] = pos[j];
    alive[j] = pos[j] < end_rel;
  }
  for (int it = 0; it < kF1Warm; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) step(pos[j], cnt[j], code[j], alive[j]);
  }
  // Compaction: finished chains write their result; survivors go to a per-wave LDS list, so phase 2
  // walks them 64 per lockstep slot instead of keeping all 256 lanes-slots busy to the chunk end.
  int* list = f1_live[wv];
  int nlive = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t mask = __ballot(alive[j]);
    if (alive[j]) {
      const int idx = nlive + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
      list[3 * idx] = lane + 64 * j;
      list[3 * idx + 1] = pos[j];
      list[3 * idx + 2] = cnt[j];
    } else {
      x[lane + 64 * j] = code[j];
      m[lane + 64 * j] = cnt[j];
    }
    nlive += __popcll(mask);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the list is visible to the whole wave
  __builtin_amdgcn_wave_barrier();
  // Few survivors (the usual case once the framing check has run): hand them to f1_chase_kernel,
  // which walks them one lane each with all lanes busy, instead of keeping this wave (and its LDS
  // stage) alive for ~chunk/record-size lockstep steps with 2-3 of 64 lanes active.
  if (nlive <= kF1Chase) {
    if (lane < nlive) {
      int32_t* o = chase + (c * kF1Chase + lane) * 3;
      o[0] = list[3 * lane];
      o[1] = list[3 * lane + 1];
      o[2] = list[3 * lane + 2];
    }
    if (lane == 0) chase_n[c] = nlive;
    return;
  }
  if (lane == 0) chase_n[c] = 0;
  // Phase 2 (many survivors): walk them here, 64 per lockstep slot.
  for (int s0 = 0; s0 < nlive; s0 += 64) {
    const int i = s0 + lane;
    bool al = i < nlive;
    int e = 0, ps = 0, ct = 0;
    if (al) {
      e = list[3 * i];
      ps = list[3 * i + 1];
      ct = list[3 * i + 2];
    }
    int cd = ps;
    while (__any(al)) step(ps, ct, cd, al);
    if (i < nlive) {
      x[e] = cd;
      m[e] = ct;
    }
  }
}

// Survivors of f1_fn_kernel, one lane each, walked to the end of their chunk straight from the
// run in global memory (the chunk's bytes are L2-resident from the stage).
__global__ void __launch_bounds__(256) f1_chase_kernel(uint8_t* const* bases, const int64_t* nbytes,
                                                       const int64_t* chunk_base, const int32_t* chunk_run,
                                                       int64_t nchunks, const int32_t* chase, const int32_t* chase_n,
                                                       int32_t* fx, int32_t* fn, int key_kind, int partial) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = t / kF1Chase;
  const int i = (int)(t % kF1Chase);
  if (c >= nchunks || i >= chase_n[c]) return;
  const int r = chunk_run[c];
  const int64_t n = nbytes[r];
  const int64_t c0 = (c - chunk_base[r]) * kF1Chunk;
  const GlobalU8* buf = (const GlobalU8*)(uintptr_t)(bases[r] + c0);
  const int end_rel = (int)min((int64_t)kF1Chunk, n - c0);
  const int lim = (int)min(n - c0, (int64_t)(kF1Chunk + kF1Halo));
  const int64_t nrel64 = n - c0;
  const int nrel = (int)min(nrel64, (int64_t)(1 << 30));
  const int32_t* in = chase + (c * kF1Chase + i) * 3;
  const int e = in[0];
  int pos = in[1], cnt = in[2], code = pos;
  bool alive = true;
  while (alive) f1_step<true>(buf, lim, nrel64, nrel, end_rel, key_kind, pos, cnt, code, alive, partial != 0);
  fx[c * kF1Entries + e] = code;
  fn[c * kF1Entries + e] = cnt;
}

__global__ void __launch_bounds__(256) f1_super_kernel(const int64_t* nbytes, const int64_t* chunk_base,
                                                       const int64_t* sup_base, const int32_t* sup_run, int64_t nsup,
                                                       const int32_t* fx, const int32_t* fn, int64_t* sx,
                                                       int64_t* sn) {
  // wave-uniform (readfirstlane: the compiler takes threadIdx.x >> 6 as divergent, and everything loaded
  // through it would be per-lane vector loads and VALU arithmetic)
  const int64_t sidx = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (sidx >= nsup) return;
  const int r = sup_run[sidx];
  const int64_t n = nbytes[r];
  const int64_t cb = chunk_base[r];
  const int64_t nch = chunk_base[r + 1] - cb;
  const int64_t first = (sidx - sup_base[r]) * kF1Super;
  const int64_t last = min(first + kF1Super, nch);
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    const int e = lane + 64 * j;
    int64_t p = first * kF1Chunk + e, cnt = 0, res;
    for (;;) {
      if (p >= n) {
        res = p;
        break;
      }
      const int64_t lc = p / kF1Chunk;
      if (lc >= last) {
        res = p;
        break;
      }
      const int64_t rel = p - lc * kF1Chunk;
      if (rel >= kF1Entries) {
        res = kSupFallback;
        break;
      }
      const int64_t slot = (cb + lc) * kF1Entries + rel;
      const int32_t x = fx[slot];
      cnt += fn[slot];
      if (x < 0) {
        res = x == kFnInvalid ? kSupInvalid : x == kFnFallback ? kSupFallback : -3 - (lc * kF1Chunk + (-1 - (int64_t)x));
        break;
      }
      p = lc * kF1Chunk + x;
    }
    sx[sidx * kF1Entries + e] = res;
    sn[sidx * kF1Entries + e] = cnt;
  }
}

__global__ void __launch_bounds__(64) f1_top_kernel(const int64_t* nbytes, const int64_t* sup_base, int nruns,
                                                    const int64_t* sx, const int64_t* sn, int64_t* sup_entry,
                                                    int64_t* sup_first, int64_t* counts, int64_t* rec_bytes,
                                                    int* status) {
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= nruns) return;
  const int64_t n = nbytes[r];
  const int64_t sb = sup_base[r];
  const int64_t span = (int64_t)kF1Super * kF1Chunk;
  int64_t p = 0, total = 0, rb = n;
  int st = 0;
  while (p < n) {
    const int64_t sidx = p / span;
    const int64_t rel = p - sidx * span;
    if (rel >= kF1Entries) {
      st = 2;
      break;
    }
    const int64_t slot = (sb + sidx) * kF1Entries + rel;
    const int64_t code = sx[slot];
    sup_entry[sb + sidx] = p;
    sup_first[sb + sidx] = total;
    total += sn[slot];
    if (code >= 0) {
      if (code <= p) {  // no progress: cannot happen on a well-formed table
        st = 1;
        break;
      }
      p = code;
      continue;
    }
    if (code == kSupInvalid) st = 1;
    else if (code == kSupFallback) st = 2;
    else rb = -3 - code;
    break;
  }
  if (st == 0 && p > n) st = 1;
  counts[r] = total;
  rec_bytes[r] = rb;
  status[r] = st;
}

__global__ void __launch_bounds__(256) f1_expand_kernel(const int64_t* nbytes, const int64_t* chunk_base,
                                                        const int64_t* sup_base, const int32_t* sup_run, int64_t nsup,
                                                        const int32_t* fx, const int32_t* fn,
                                                        const int64_t* sup_entry, const int* status,
                                                        int64_t* ck_start, int64_t* ck_count) {
  const int64_t sidx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (sidx >= nsup) return;
  const int r = sup_run[sidx];
  if (status[r] != 0) return;  // re-indexed by the serial scan (or corrupt)
  const int64_t n = nbytes[r];
  const int64_t cb = chunk_base[r];
  const int64_t nch = chunk_base[r + 1] - cb;
  const int64_t first = (sidx - sup_base[r]) * kF1Super;
  const int64_t last = min(first + kF1Super, nch);
  int64_t p = sup_entry[sidx];
  for (int64_t lc = first; lc < last; ++lc) {
    const int64_t cg = cb + lc;
    const int64_t rel = p - lc * kF1Chunk;
    if (p < 0 || p >= n || rel >= kF1Chunk || rel >= kF1Entries || rel < 0) {
      ck_start[cg] = p < 0 ? 0 : p;
      ck_count[cg] = 0;
      continue;
    }
    const int64_t slot = cg * kF1Entries + rel;
    const int32_t x = fx[slot];
    ck_start[cg] = p;
    ck_count[cg] = fn[slot];
    p = x < 0 ? -1 : lc * kF1Chunk + x;
  }
}

// Pass 2, one lane per chunk: the chunk's records are walked straight from memory (each lane streams
// its own 4 KiB chunk through the caches), so 64 chunks progress per wave instead of one.
// (Folding F2 into this walk was measured slower: 13.7 vs 11.6 ms for the 2 GB secondary sort. Each
// lane then scatters 48 bytes per record into five arrays, while normalize_kernel's stores coalesce.)
__global__ void __launch_bounds__(256) f1_index_lane_kernel(uint8_t* const* bases, const int64_t* nbytes,
                                                            const int64_t* chunk_base, const int32_t* chunk_run,
                                                            const int64_t* ck_start, const int64_t* ck_count,
                                                            const int64_t* ck_ord, const int64_t* elem_off,
                                                            const int64_t* rec_bytes, int64_t* const* offsets,
                                                            int64_t total_chunks) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= total_chunks) return;
  const int r = chunk_run[c];
  const int64_t here = ck_count[c];
  const int64_t n = nbytes[r];
  const uint8_t* p = bases[r];
  int64_t* out = offsets[r] + (ck_ord[c] - elem_off[r]);
  int64_t pos = ck_start[c];
  for (int64_t i = 0; i < here; ++i) {
    out[i] = pos;
    int64_t kl = 0, vl = 0;
    const int a = vint_decode(p + pos, (size_t)(n - pos), &kl);
    const int b = vint_decode(p + pos + a, (size_t)(n - pos - a), &vl);
    pos += a + b + kl + vl;
  }
  if (c == chunk_base[r]) offsets[r][elem_off[r + 1] - elem_off[r]] = rec_bytes[r];
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
  // one unaligned 8-byte load when the content has 8 bytes (the byte loop costs 8 load instructions)
  typedef uint64_t __attribute__((aligned(1))) u64_u;
  e.hi = cl >= 8 ? __builtin_bswap64(*reinterpret_cast<const u64_u*>(key + o)) : load_be_prefix(key + o, cl);
  const uint64_t capped = cl > 0xFFFF ? 0xFFFF : (uint64_t)cl;
  e.lo = (capped << 48) | (uint64_t)g;
  out[g] = e;
  ctx.keyptr[g] = key + o;
  ctx.keylen[g] = cl;
  ctx.recptr[g] = rec;
  ctx.reclen[g] = (int32_t)(ctx.offsets[r][pos + 1] - ctx.offsets[r][pos]);
}

__global__ void __launch_bounds__(256) record_sizes_kernel(GenericKeyCtx ctx, const Elem* elems, int64_t n,
                                                           int64_t* sizes) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sizes[i] = ctx.reclen[elems[i].lo & 0xFFFFFFFFFFFFull];
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
// One lane per record (in merged order). Records are byte-aligned anywhere, so the copy uses
// unaligned 16-byte accesses (legal for global memory on gfx950; the compiler emits the same for a
// 16-byte memcpy): a record of L >= 16 bytes moves as ceil(L/16) chunks, the last one shifted back
// to end at L (it overlaps its predecessor and rewrites the same bytes). Up to 8 chunks (128 bytes)
// are loaded before the first is stored, and loads and stores are unguarded (offsets clamped):
// guarded stores would each wait for every earlier store, since stores count in vmcnt on CDNA.
__device__ __forceinline__ void copy_small(const uint8_t* s, uint8_t* d, int L) {
  if (L >= 8) {
    uint64_t a, b;
    __builtin_memcpy(&a, s, 8);
    __builtin_memcpy(&b, s + L - 8, 8);
    __builtin_memcpy(d, &a, 8);
    __builtin_memcpy(d + L - 8, &b, 8);
  } else if (L >= 4) {
    uint32_t a, b;
    __builtin_memcpy(&a, s, 4);
    __builtin_memcpy(&b, s + L - 4, 4);
    __builtin_memcpy(d, &a, 4);
    __builtin_memcpy(d + L - 4, &b, 4);
  } else if (L >= 2) {
    uint16_t a, b;
    __builtin_memcpy(&a, s, 2);
    __builtin_memcpy(&b, s + L - 2, 2);
    __builtin_memcpy(d, &a, 2);
    __builtin_memcpy(d + L - 2, &b, 2);
  } else if (L == 1) {
    d[0] = s[0];
  }
}

// F4 with kGatherLanes lanes per record: the lanes of a group copy 16-byte pieces of one record, so a
// wave's load touches 64 / kGatherLanes records (two or three cache lines each) instead of 64, and
// consecutive groups write consecutive output records. Pieces past the record end are clamped to its
// last 16 bytes (overlapping stores of identical bytes). 2 GB secondary sort: the merge takes 0.8 ms less
// than with one lane per record (2.2 ms gather); 4 lanes per record measured the same as 8.
template <int kGatherLanes>
__global__ void __launch_bounds__(256) gather_var_grp_kernel(GenericKeyCtx ctx, const Elem* elems, int64_t n,
                                                             const int64_t* out_off, uint8_t* out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kGatherLanes;
  const int sub = (int)(threadIdx.x % kGatherLanes);
  if (i >= n) return;
  const uint64_t g = elems[i].lo & 0xFFFFFFFFFFFFull;
  const uint8_t* src = ctx.recptr[g];
  const int L = ctx.reclen[g];
  uint8_t* dst = out + out_off[i];
  if (L < 16) {
    if (sub == 0) copy_small(src, dst, L);
    return;
  }
  constexpr int kStep = kGatherLanes * 16;
  for (int base = sub * 16; base < L; base += 2 * kStep) {
    const int o0 = min(base, L - 16);
    const int o1 = min(base + kStep, L - 16);
    const u32x4 v0 = *reinterpret_cast<const u32x4_u*>(src + o0);
    const u32x4 v1 = *reinterpret_cast<const u32x4_u*>(src + o1);
    *reinterpret_cast<u32x4_u*>(dst + o0) = v0;
    if (base + kStep < L) *reinterpret_cast<u32x4_u*>(dst + o1) = v1;
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

// Max of n int32 (record lengths), four per 16-byte load, four loads in flight per lane; one atomic
// per block (same-address atomics serialize in L2: one per wave cost ~80 us for 16M lengths).
__global__ void __launch_bounds__(256) max_i32_kernel(const int32_t* v, int64_t n, unsigned int* out) {
  __shared__ unsigned int wmax[4];
  unsigned int m = 0;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const u32x4_u* v4 = reinterpret_cast<const u32x4_u*>(v);  // v need not be 16-byte aligned
  int64_t i = t;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const u32x4 a = v4[i], b = v4[i + stride], c = v4[i + 2 * stride], d = v4[i + 3 * stride];
    const u32x4 x = __builtin_elementwise_max(__builtin_elementwise_max(a, b), __builtin_elementwise_max(c, d));
    m = max(m, max(max(x[0], x[1]), max(x[2], x[3])));
  }
  for (; i < n4; i += stride) {
    const u32x4 x = v4[i];
    m = max(m, max(max(x[0], x[1]), max(x[2], x[3])));
  }
  for (int64_t k = n4 * 4 + t; k < n; k += stride) m = max(m, (unsigned int)v[k]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, off, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3])));
}

void launch_max_i32(const int32_t* v, int64_t n, unsigned int* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(unsigned int), s);
  if (n <= 0) return;
  int64_t blocks = (n / 16 + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(max_i32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, v, n, out);
}

void launch_max_i64(const int64_t* v, int64_t n, unsigned long long* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(max_kernel, dim3((unsigned)blocks), dim3(256), 0, s, v, n, out);
}

void launch_f1_scan(uint8_t* const* bases, const int64_t* nbytes, int nruns, const int64_t* chunk_base,
                    int64_t* ck_start, int64_t* ck_count, int64_t* counts, int64_t* rec_bytes, int* status,
                    hipStream_t s, uint64_t* prof, const int* run_ids, bool partial) {
  if (nruns <= 0) return;
  if (prof)
    hipLaunchKernelGGL(f1_scan_kernel<true>, dim3((unsigned)nruns), dim3(kF1Lanes), 0, s, bases, nbytes, chunk_base,
                       ck_start, ck_count, counts, rec_bytes, status, prof, run_ids, (int)partial);
  else
    hipLaunchKernelGGL(f1_scan_kernel<false>, dim3((unsigned)nruns), dim3(kF1Lanes), 0, s, bases, nbytes,
                       chunk_base, ck_start, ck_count, counts, rec_bytes, status, prof, run_ids, (int)partial);
}

size_t f1_parallel_workspace(int64_t nchunks, int64_t nsup) {
  return (size_t)nchunks * kF1Entries * 8 + (size_t)nsup * (kF1Entries * 16 + 16) + 256 +
         (size_t)nchunks * (kF1Chase * 3 + 1) * 4 + 256;
}
int64_t f1_super_chunks() { return kF1Super; }

void launch_f1_parallel(uint8_t* const* bases, const int64_t* nbytes, int nruns, const int64_t* chunk_base,
                        const int32_t* chunk_run, int64_t nchunks, const int64_t* sup_base, const int32_t* sup_run,
                        int64_t nsup, void* workspace, int64_t* ck_start, int64_t* ck_count, int64_t* counts,
                        int64_t* rec_bytes, int* status, hipStream_t s, int key_kind, bool partial) {
  if (nruns <= 0) return;
  uint8_t* w = static_cast<uint8_t*>(workspace);
  int32_t* fx = reinterpret_cast<int32_t*>(w);
  int32_t* fn = fx + nchunks * kF1Entries;
  int64_t* sx = reinterpret_cast<int64_t*>(fn + nchunks * kF1Entries);
  int64_t* sn = sx + nsup * kF1Entries;
  int64_t* sup_entry = sn + nsup * kF1Entries;
  int64_t* sup_first = sup_entry + nsup;
  int32_t* chase = reinterpret_cast<int32_t*>(sup_first + nsup + 32);
  int32_t* chase_n = chase + nchunks * kF1Chase * 3;
  if (nchunks > 0) {
    hipLaunchKernelGGL(f1_fn_kernel, dim3((unsigned)((nchunks + kF1FnWaves - 1) / kF1FnWaves)), dim3(64 * kF1FnWaves),
                       0, s, bases, nbytes, chunk_base, chunk_run, nchunks, fx, fn, key_kind, chase, chase_n,
                       (int)partial);
    const int64_t lanes = nchunks * kF1Chase;
    hipLaunchKernelGGL(f1_chase_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, bases, nbytes,
                       chunk_base, chunk_run, nchunks, chase, chase_n, fx, fn, key_kind, (int)partial);
    hipLaunchKernelGGL(f1_super_kernel, dim3((unsigned)((nsup + 3) / 4)), dim3(256), 0, s, nbytes, chunk_base,
                       sup_base, sup_run, nsup, fx, fn, sx, sn);
    (void)hipMemsetAsync(sup_entry, 0xFF, (size_t)nsup * 8, s);
  }
  hipLaunchKernelGGL(f1_top_kernel, dim3((unsigned)((nruns + 63) / 64)), dim3(64), 0, s, nbytes, sup_base, nruns,
                     sx, sn, sup_entry, sup_first, counts, rec_bytes, status);
  if (nchunks > 0)
    hipLaunchKernelGGL(f1_expand_kernel, dim3((unsigned)((nsup + 255) / 256)), dim3(256), 0, s, nbytes, chunk_base,
                       sup_base, sup_run, nsup, fx, fn, sup_entry, status, ck_start, ck_count);
}

void launch_f1_index(uint8_t* const* bases, const int64_t* nbytes, const int64_t* chunk_base,
                     const int32_t* chunk_run, const int64_t* ck_start, const int64_t* ck_count,
                     const int64_t* ck_ord, const int64_t* elem_off, const int64_t* rec_bytes,
                     int64_t* const* offsets, int64_t total_chunks, hipStream_t s) {
  if (total_chunks <= 0) return;
  hipLaunchKernelGGL(f1_index_lane_kernel, dim3((unsigned)((total_chunks + 255) / 256)), dim3(256), 0, s, bases,
                     nbytes, chunk_base, chunk_run, ck_start, ck_count, ck_ord, elem_off, rec_bytes, offsets,
                     total_chunks);
}

int64_t f1_chunk_bytes() { return kF1Chunk; }

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
  // 8 lanes per record (one record per lane measured 0.8 ms slower on the 2 GB secondary sort)
  hipLaunchKernelGGL(gather_var_grp_kernel<8>, dim3((unsigned)((n * 8 + 255) / 256)), dim3(256), 0, s, ctx, elems, n,
                     out_off, out);
}

void launch_buffer_cuts(const int64_t* out_off, int64_t n, int64_t chunk, int64_t nbuf, int64_t* cuts,
                        hipStream_t s) {
  hipLaunchKernelGGL(buffer_cuts_kernel, dim3((unsigned)((nbuf + 1 + 255) / 256)), dim3(256), 0, s, out_off, n,
                     chunk, nbuf, cuts);
}

}  // namespace gpu
}  // namespace uda
