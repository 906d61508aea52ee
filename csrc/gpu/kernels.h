// Host-callable launchers for the gfx950 HIP kernels of the shuffle/merge data path.
//
// Every launcher takes raw device pointers and a hipStream_t and never allocates or synchronizes,
// so a sequence of launches can be enqueued from one host thread (or captured into a hipGraph).
//
// Map to the reference's CPU hot loops:
//   F1 record index        -> index_records_serial / verify_fixed_stride
//   F2 key normalization   -> extract_keys_fixed / extract_keys_generic (+ __device__ compare)
//   F3 k-way merge         -> merge_partition + merge_pass (pairwise merge-path tree on keys)
//   F4 serialize / gather  -> gather_fixed / gather_var + buffer cut points
//   F6 block decompress    -> snappy_decompress_blocks / lzo1x_decompress_blocks
// plus TeraGen-shaped synthetic map-output generation and device-side validation.
#pragma once
#include "uda/hash.h"
#include <hip/hip_runtime.h>

#include <cstdint>

namespace uda {
namespace gpu {

// 16-byte merge element. Ordering is lexicographic on (hi, lo).
//   FIXED10 mode: hi = key bytes 0..7 (big-endian), lo = key bytes 8..9 << 48 | run << 32 | pos.
//   GENERIC mode: hi = content prefix bytes 0..7, lo = global record ordinal (ties resolved
//                 with a full-key comparison through the record index; see merge.hip).
struct alignas(16) Elem {
  uint64_t hi;
  uint64_t lo;
};

// TeraSort record geometry: Text key (VInt 10 + 10 bytes) and Text value (VInt 90 + 90 bytes)
// inside an IFile record (VInt keyLen=11, VInt valLen=91): 104 bytes, 8-byte aligned.
constexpr int kTeraKeyBytes = 10;
constexpr int kTeraValBytes = 90;
constexpr int kTeraRecordBytes = 104;
constexpr int kTeraKeyOffset = 3;  // [0x0B][0x5B][0x0A] key...

// Descriptor of a sorted run (one map-output partition slice) living in device memory.
struct RunDesc {
  const uint8_t* base;  // first record
  int64_t nrec;         // records in the run
  int64_t nbytes;       // bytes (records only, no EOF marker)
  const int64_t* offsets;  // GENERIC: record start offsets relative to base (nrec+1 entries), or null
};

// ---------------------------------------------------------------- synthetic data (TeraGen)
// Fill `nruns` runs; run r has `nrec[r]` records written at `bases[r]` (8-byte aligned) with keys
// whose first 8 bytes lie in [key_lo[r], key_lo[r] + key_span[r]) in ascending order (stratified
// with random jitter, so the K runs of one reducer interleave randomly), random 2 trailing key
// bytes and 90 printable value bytes, followed by the 2-byte EOF marker. Accumulates an
// order-independent checksum (sum of record_hash) per run into `run_checksum[r]` (zero it first).
// unsorted != 0: keys uniform in the same range in generation order (a map task's input before its
// sort; launch_sort_fixed_run turns each run into a sorted map-output partition).
void launch_teragen(uint8_t* const* bases, const int64_t* nrec, const uint64_t* key_lo,
                    const uint64_t* key_span, const uint64_t* seeds, int nruns, int64_t max_nrec,
                    unsigned long long* run_checksum, hipStream_t s, int unsorted = 0);

// ---------------------------------------------------------------- F8 map-side sort (radix.hip)
// Sort the n TeraSort records at `base` by their 10-byte key (stable LSD radix sort, 8-bit digits,
// then one record gather). `ws` holds sort_fixed_ws_bytes(n) bytes of device memory; n < 2^32.
// staged: the unsorted records were written to sort_fixed_ws_records(ws, n) instead (no copy aside);
// the sorted run lands at `base` followed by the IFile EOF marker.
int64_t sort_fixed_ws_bytes(int64_t n);
uint8_t* sort_fixed_ws_records(void* ws, int64_t n);
void launch_sort_fixed_run(uint8_t* base, int64_t n, void* ws, hipStream_t s, bool staged = false);

// ---------------------------------------------------------------- round splitting
// For each (run r, boundary b): out[r*(nb+2) + 1 + b] = lower_bound of boundary key (hi, lo16)
// inside run r (FIXED10 layout); out[r*(nb+2)] = 0 and out[r*(nb+2)+nb+1] = nrec[r].
void launch_split_fixed(uint8_t* const* bases, const int64_t* nrec, const Elem* bounds,
                        const int* run_bound_set, int nruns, int nb, int64_t* out, hipStream_t s);

// Sample every `every`-th key of each FIXED10 run (starting at every/2): run r writes its samples
// at out[sample_off[r] ...] as Elem{hi, lo16 << 48}.
void launch_sample_fixed(uint8_t* const* bases, const int64_t* nrec, int nruns, int64_t every,
                         const int64_t* sample_off, int64_t total, Elem* out, hipStream_t s);

// Block first-key index of block-compressed FIXED10 streams: for every block b, the key of the first
// record that starts in it, read from its decoded prefix at prefix + b * slot + first_off[b] (-1: none:
// Elem{~0, ~0}). *bad |= 1 when a record there is not the TeraSort layout.
void launch_block_first_keys(const uint8_t* prefix, int64_t slot, const int32_t* first_off, int n, Elem* out, int* bad,
                             hipStream_t s);

// ---------------------------------------------------------------- key extraction (F2)
// Build Elem keys for all records of `nruns` FIXED10 runs; run r's elements start at
// elem_off[r]. Sets *bad_layout to 1 if any record header is not the TeraSort layout.
void launch_extract_fixed(const RunDesc* runs, const int64_t* elem_off, int nruns, int64_t total,
                          Elem* out, int* bad_layout, hipStream_t s);

// ---------------------------------------------------------------- merge tree (F3)
constexpr int kMergeTile = 2048;         // FIXED10: output elements per workgroup (256 threads x 8)
constexpr int kGenericMergeTile = 1024;  // GENERIC: smaller tiles leave LDS for the staged key bytes
// One merge pass. Pair p merges the adjacent sorted element ranges A = [pairs[3p], pairs[3p+1]) and
// B = [pairs[3p+1], pairs[3p+2]) into the same index range of the output (B may be empty: the range
// is copied through). Pair p produces tiles [tile_prefix[p], tile_prefix[p+1]) of kMergeTile
// outputs each (the last tile of a pair may be short). Pairs are planned on the host
// (merge_plan.h) so that segments of different groups (reducers) never merge.
struct PassDesc {
  const int64_t* pairs;        // 3 * npairs entries
  const int64_t* tile_prefix;  // npairs + 1 entries
  int npairs;
  int ntiles;
};
// splits[t] = merge-path split (elements taken from A) at the first output of tile t.
void launch_merge_partition(const Elem* in, PassDesc pd, int64_t* splits, hipStream_t s);
void launch_merge_pass(const Elem* in, Elem* out, PassDesc pd, const int64_t* splits, hipStream_t s);

// GENERIC key context. Record i of run r starts at bases[r] + offsets[r][i]; kind = uda::KeyKind.
// After F2 every record g (global ordinal, run-major) also has direct side tables so the merge and
// the gather never re-parse headers: key content pointer/length and record pointer/length.
// GENERIC Elem: hi = first 8 content bytes (big-endian), lo = min(content_len, 0xFFFF) << 48 | g.
struct GenericKeyCtx {
  uint8_t* const* bases;
  const int64_t* const* offsets;
  int kind;
  const uint8_t** keyptr;   // [g] key content
  int32_t* keylen;          // [g] content length
  const uint8_t** recptr;   // [g] record start
  int32_t* reclen;          // [g] record size
};
void launch_merge_partition_generic(const Elem* in, PassDesc pd, int64_t* splits, GenericKeyCtx ctx,
                                    hipStream_t s);
void launch_merge_pass_generic(const Elem* in, Elem* out, PassDesc pd, const int64_t* splits,
                               GenericKeyCtx ctx, hipStream_t s);

// ---------------------------------------------------------------- single-pass K-way merge, generic keys
constexpr int kGkMaxRuns = 128;  // runs per merge on the generic single-pass path
int generic_kway_cap();          // elements per cell
// samples[soff[r] + j] = cur[eoff[r] + j * step + step / 2]
void launch_gk_sample(const Elem* cur, const int64_t* eoff, const int64_t* soff, int K, int64_t step, int64_t ns,
                      Elem* out, hipStream_t s);
void launch_gk_pick(const Elem* merged, int64_t ns, int64_t C, Elem* bounds, hipStream_t s);
// split[r * (C + 1) + j] = first element of run r not below splitter j - 1 (0 / run length at the
// ends), from a histogram of the merged samples by run (hist: K * C ints of scratch).
// eoff: element offsets of the runs at this level; ord_off: run boundaries in record ordinals.
void launch_gk_split_hist(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff, const int64_t* ord_off,
                          const Elem* merged, int64_t ns, const int64_t* soff, int64_t step, int K, const Elem* bounds,
                          int64_t C, int* hist, int64_t* split, hipStream_t s);
// Cells [c_first, c_first + c_count) of C.
void launch_gk_cells(GenericKeyCtx ctx, const Elem* cur, const int64_t* eoff, int K, const int64_t* split, int64_t C,
                     int64_t c_first, int64_t c_count, Elem* out, int* overflow, hipStream_t s);
// For each of nb cell boundaries cb[i]: merged elements and record bytes before it.
void launch_gk_round_bounds(const int64_t* split, int K, int64_t C, const int64_t* cb, int nb,
                            const int64_t* const* rec_off, int64_t* elem, int64_t* bytes, hipStream_t s);

// ---------------------------------------------------------------- single-pass K-way merge (F2+F3+F4)
constexpr int kKwCap = 2048;       // records per cell (LDS capacity of one workgroup)
constexpr int kKwMaxRuns = 256;    // runs per group on the single-pass path (8 GPUs x 32 maps)
struct KwayDesc {
  const RunDesc* runs;        // every run of the round, grouped by reducer
  const int* group_first;     // G+1
  const int64_t* cell_first;  // G+1: first cell (workgroup) of each group
  const int64_t* split;       // [run][nbmax+2]: split[r*(nbmax+2) + c] = first record of cell c in run r
  int nbmax;
  const int64_t* group_out;   // G: first output record of each group
  int G;
  int* overflow;              // cells merged by the wave-level PQ (did not fit LDS)
  int* bad_layout;            // set if a record is not TeraSort-shaped
  int cap = kKwCap;           // records per cell on the LDS path (kway_cap_supported)
  unsigned long long* prof = nullptr;  // optional [cell][5] phase timestamps (UDA_KWAY_PROF)
  int kmax = kKwMaxRuns;      // most runs in one group of this plan (sizes the per-slice LDS tables)
  int staged = 0;             // records staged in LDS once (kway_staged_kernel; cap 512 or 1024)
};
// bounds[g*nbmax + j] = splitter j of group g (sample (j+1)*ns_g/C_g of the group's merged samples),
// +infinity for j >= C_g - 1.
void launch_pick_splitters(const Elem* samples, const int64_t* gsamp_off, const int64_t* gcells, int G, int nbmax,
                           Elem* bounds, hipStream_t s);
void launch_kway_tiles(const KwayDesc& kd, int64_t ncells, uint8_t* out, hipStream_t s);
int kway_cap_supported(int cap);
// split[r][c] for the k-way cells, bracketed by the run's own regular sample (soff / every as given
// to launch_sample_fixed; samples in per-run order, not merged).
void launch_split_sampled(uint8_t* const* bases, const int64_t* nrec, const Elem* samples, const int64_t* soff,
                          int64_t every, const Elem* bounds, const int* run_bound_set, int nruns, int nb, int64_t* out,
                          hipStream_t s);

// ---------------------------------------------------------------- GENERIC record path (F1/F2/F4)
// F1 pass 1 (one wave per run): chunk checkpoints ck_start/ck_count for the chunks of run r at
// [chunk_base[r], chunk_base[r+1]) (chunks of f1_chunk_bytes()), records per run, record bytes
// before the EOF marker, status != 0 on a corrupt/truncated stream. prof: diagnostic cycle split.
// partial: every run is the landed prefix of a stream still arriving; a record cut by its end ends
// the run like the EOF marker, so rec_bytes is the end of its last complete record.
int64_t f1_chunk_bytes();
void launch_f1_scan(uint8_t* const* bases, const int64_t* nbytes, int nruns, const int64_t* chunk_base,
                    int64_t* ck_start, int64_t* ck_count, int64_t* counts, int64_t* rec_bytes, int* status,
                    hipStream_t s, uint64_t* prof = nullptr, const int* run_ids = nullptr, bool partial = false);
// F1 pass 1, parallel form: same outputs as launch_f1_scan from per-chunk transfer functions
// composed per superchunk (f1_super_chunks() chunks) and per run. sup_base[r]..sup_base[r+1] are
// run r's superchunks, sup_run their run. status[r] == 2: the run needs the serial scan.
size_t f1_parallel_workspace(int64_t nchunks, int64_t nsup);
int64_t f1_super_chunks();
void launch_f1_parallel(uint8_t* const* bases, const int64_t* nbytes, int nruns, const int64_t* chunk_base,
                        const int32_t* chunk_run, int64_t nchunks, const int64_t* sup_base, const int32_t* sup_run,
                        int64_t nsup, void* workspace, int64_t* ck_start, int64_t* ck_count, int64_t* counts,
                        int64_t* rec_bytes, int* status, hipStream_t s, int key_kind = -1, bool partial = false);
// F1 pass 2 (one wave per chunk): record offsets; ck_ord = exclusive scan of ck_count (global
// record ordinal of each chunk's first record), elem_off = first ordinal of each run (nruns+1),
// chunk_run[c] = run of chunk c. offsets[r] has counts[r]+1 entries (last = record bytes).
void launch_f1_index(uint8_t* const* bases, const int64_t* nbytes, const int64_t* chunk_base,
                     const int32_t* chunk_run, const int64_t* ck_start, const int64_t* ck_count,
                     const int64_t* ck_ord, const int64_t* elem_off, const int64_t* rec_bytes,
                     int64_t* const* offsets, int64_t total_chunks, hipStream_t s);
// F2: normalized elements for all records; elem_off[r] = first element of run r (nruns+1 entries).
void launch_normalize_generic(GenericKeyCtx ctx, const int64_t* elem_off, int nruns, int64_t total, Elem* out,
                              hipStream_t s);
// F4: sizes[i] = size of the record elems[i] refers to.
void launch_record_sizes(GenericKeyCtx ctx, const Elem* elems, int64_t n, int64_t* sizes, hipStream_t s);
// Exclusive scan of n int64 (out has n+1 entries, out[n] = total); tmp >= scan_tmp_elems(n).
int64_t scan_tmp_elems(int64_t n);
void launch_exclusive_scan(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s);
// F4: copy record elems[i] to out + out_off[i].
void launch_gather_var(GenericKeyCtx ctx, const Elem* elems, int64_t n, const int64_t* out_off, uint8_t* out,
                       hipStream_t s);
// *out = max(v[0..n)) (zeroed first).
void launch_max_i64(const int64_t* v, int64_t n, unsigned long long* out, hipStream_t s);
// *out = max of n non-negative int32.
void launch_max_i32(const int32_t* v, int64_t n, unsigned int* out, hipStream_t s);
// Delivery cut points: cuts[j] = output byte offset of the first record whose offset >= j*chunk
// (cuts[nbuf] = total bytes), j = 0..nbuf.
void launch_buffer_cuts(const int64_t* out_off, int64_t n, int64_t chunk, int64_t nbuf, int64_t* cuts,
                        hipStream_t s);

// ---------------------------------------------------------------- gather / serialize (F4)
// out[i*104 .. +104) = record of elem[i] (FIXED10: run/pos encoded in elem.lo).
void launch_gather_fixed(const Elem* elems, int64_t n, uint8_t* const* run_bases, uint8_t* out,
                         hipStream_t s);

// ---------------------------------------------------------------- batched copy
struct CopyDesc {
  const uint8_t* src;
  uint8_t* dst;
  int64_t bytes;
};
// descs: device array of n descriptors; max_bytes: largest descriptor (sizes the grid).
void launch_batched_copy(const CopyDesc* descs, int n, int64_t max_bytes, hipStream_t s, int max_blocks = 2048);

// ---------------------------------------------------------------- block decode (F6)
// One Hadoop compressed block: chunks [u32 BE clen][clen bytes]... in [src, src_end) of the
// compressed buffer decode to exactly `raw` bytes at dst of the output buffer.
struct DecodeDesc {
  int64_t src;
  int64_t src_end;
  int64_t dst;
  int64_t raw;
};
// codec: 1 = Snappy, 2 = LZO1X (uda::Codec values). *status |= 1 if any block is corrupt.
// clip > 0: prefix decode, only the first `clip` raw bytes of every block are produced (at its dst).
void launch_block_decode(int codec, const uint8_t* in, uint8_t* out, const DecodeDesc* descs, int n, int* status,
                         hipStream_t s, int64_t clip = 0);
// The LZO lane kernel's per-block decode on the host (tests without a GPU).
bool lzo_lane_decode_host(const uint8_t* in, int64_t n, uint8_t* out, int64_t out_cap, int64_t* out_len);
// Framing walk of device-resident streams (one lane per stream). out == nullptr: per-stream block
// counts and raw bytes; else the descriptors with absolute src addresses (decode with in = nullptr).
// status[s] = 1: framing not resolvable without decoding (zero status first).
void launch_frame_streams(const uint8_t* const* ptrs, const int64_t* lens, int nstreams, int codec,
                          const int64_t* desc_first, const int64_t* raw_first, int64_t* nblocks, int64_t* raw,
                          DecodeDesc* out, int* status, hipStream_t s);

// ---------------------------------------------------------------- validation
// Checks key order of `n` FIXED10 records at `recs` (and against *prev_key if has_prev) and
// accumulates an order-independent checksum. Results: stats[0] += out-of-order count,
// stats[1] += checksum (and *group_ck += checksum when given). Writes the last key to *last_key.
void launch_validate_fixed(const uint8_t* recs, int64_t n, const Elem* prev_key, int has_prev,
                           Elem* last_key, unsigned long long* stats, hipStream_t s,
                           unsigned long long* group_ck = nullptr);

// out[i] = sum of record hashes of FIXED10 slice runs[i] (device array of n RunDesc; out zeroed
// here). max_nrec sizes the grid.
void launch_slice_checksums(const RunDesc* runs, int n, int64_t max_nrec, unsigned long long* out, hipStream_t s);
// *bad = 1 if any record of the n runs is not TeraSort-shaped (FIXED10 header check).
void launch_check_fixed(const RunDesc* runs, int n, int64_t max_nrec, int* bad, hipStream_t s);
// *errors += number of i with a[i] != b[i].
void launch_count_mismatch(const unsigned long long* a, const unsigned long long* b, int n,
                           unsigned long long* errors, hipStream_t s);

// Order-independent checksums: shared with the host (uda/hash.h).
using ::uda::mix64;
using ::uda::record_hash;

}  // namespace gpu
}  // namespace uda
