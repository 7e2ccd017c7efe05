// rr_internal.h — launchers shared between the C-ABI host code (rr_api.cpp) and the HIP kernels
// (rr_kernels.hip). Not part of the public ABI (see include/rag_retrieval.h).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace rr {

// Fused kernel geometry: 8 waves per workgroup (2 per SIMD), each wave owns a 32-document tile at a
// time; 32 query slots per pass (the N dimension of the 32x32 MFMA).
constexpr int kWaves      = 8;
constexpr int kThreads    = kWaves * 64;
constexpr int kQSlots     = 32;
constexpr int kTileDocs   = 32;
constexpr int kGroupChunks = 8;   // 16-byte loads per lane kept in flight per pipeline stage

// Kernel data types (how a corpus dtype is stored and multiplied).
//   KDT_F32_MFMA : fp32 rows, v_mfma_f32_32x32x2_f32 (a plain fmaf chain per score)
//   KDT_BF16     : bf16 rows, v_mfma_f32_32x32x16_bf16 against the query's bf16 hi + lo
//   KDT_F32_SPLIT: fp32 rows stored as f16 hi + lo (per-row power-of-two scale; x = (hi + lo) * 2^-e
//                  to 2^-22 relative), 3 x v_mfma_f32_32x32x16_f16 per chunk (hi*qhi + hi*qlo + lo*qhi)
constexpr int KDT_F32_MFMA = 0;
constexpr int KDT_BF16 = 1;
constexpr int KDT_F32_SPLIT = 2;
//   KDT_F32_X3   : fp32 rows, each value split exactly into three bf16 in registers, 6 bf16 MFMAs
//                  (split-K kernel only; rr_sk.hip)
constexpr int KDT_F32_X3 = 3;
//   KDT_SCREEN   : fp32 rows read as f16 against the query's f16 hi + lo: an upper bound of the KDT_F32_X3
//                  score for the screened search (split-K kernel only; rr_sk.hip "Screened search")
constexpr int KDT_SCREEN = 6;
//   KDT_SCREEN16 : the same screen over an f16 copy of the fp32 rows (the values KDT_SCREEN rounds to in
//                  registers, stored: half the bytes per screened search; rr_sk.hip DT 7)
constexpr int KDT_SCREEN16 = 7;
//   KDT_SCREEN8  : the screen over an int8 copy (per-row scale, per-row error norm; a quarter of the fp32 bytes)
//                  against the query's two int8 pieces, v_mfma_i32_32x32x32_i8 (rr_sk.hip DT 8)
constexpr int KDT_SCREEN8 = 8;
//   KDT_SCREEN9  : the int8 screen for bf16 storage: an int8 copy of the bf16 rows against ONE int8 piece per query, so
//                  64 query slots fit one pass (rr_sk.hip DT 9); verified with the bf16 kernel's own arithmetic
constexpr int KDT_SCREEN9 = 9;

// Smallest fused-kernel list width KT >= k (4, 8, 16, 32); 0 if k > RR_FUSED_KMAX.
int fused_kt(int k);

// Dynamic LDS bytes the fused kernel needs for (d, KT, kernel dtype), without the per-doc segments.
size_t fused_lds_bytes(int d, int kt, int kdt);

// Fused similarity + per-workgroup top-KT. queries: [b][d] fp32 (b <= 32) on device.
// corpus: [n][...] in the kernel dtype's storage. norms: [n] |d| (cosine). rscale: [n] split-f16 row
// scales. cand: [grid][32][KT] uint64 keys (see key encoding in rr_kernels.hip).
hipError_t launch_fused(int kdt, int metric, int kt, int grid, const void* corpus, const float* norms,
                        const float* rscale, const float* queries, int64_t n, int d, int b, uint32_t idx_base,
                        uint64_t* cand, hipStream_t s);

// Chunk geometry of a split-K launch over T tiles (32 kernel rows each) and `grid` statically scheduled workgroups:
// chunks of ct tiles, then (ct > 2, guided) the last ~2 grid tiles in 2-tile chunks, so the launch's last chunks are
// short (rr_sk.hip "Guided tail"). Shared by the kernel and the host (the repair pass maps the screen's chunks to rows).
struct ChunkGeo {
  int64_t T, T1, C1, C;
  int ct, ct2;
};
__host__ __device__ inline ChunkGeo chunk_geo(int64_t T, int ct, int64_t grid, bool guided) {
  ChunkGeo g;
  g.T = T;
  g.ct = ct;
  g.ct2 = ct > 2 ? 2 : ct;
  g.T1 = ct > 2 && T > 2 * grid && guided ? (T - 2 * grid) / ct * ct : 0;   // tiles in ct-tile chunks
  g.C1 = g.T1 / ct;
  g.C = g.C1 + (T - g.T1 + g.ct2 - 1) / g.ct2;
  return g;
}
__host__ __device__ inline int64_t chunk_tile0(const ChunkGeo& g, int64_t c) {
  return c < g.C1 ? c * g.ct : g.T1 + (c - g.C1) * g.ct2;
}
__host__ __device__ inline int chunk_ntiles(const ChunkGeo& g, int64_t c) {
  if (c < g.C1) return g.ct;
  const int64_t left = g.T - chunk_tile0(g, c);
  return (int)(left < g.ct2 ? left : g.ct2);
}

// Arguments of the split-K kernel (rr_sk.hip), all modes.
struct SkArgs {
  const char* corpus;      // this shard's rows in the storage layout
  const float* norms;      // [rows] |row| (cosine; and the screen's bound)
  const float* rscale;     // [rows] split-f16 row scales
  const float* queries;    // [slots][d] fp32
  int64_t n;               // rows of this shard
  int d, b;                // dimension, queries in this block
  uint32_t idx_base;       // global index of local row 0
  uint64_t* out;           // MODE 0: [grid][slots][KT] candidate keys
  uint64_t* clear_word;    // MODE 0 (may be null): zeroed by workgroup 0 — the exchanged flag word the block's verify
                           // raises (an earlier search with wider lists may have left keys at its position)
  uint32_t* ctr;           // MODE 0, dyn: the shard's chunk counter (0 between launches; the kernel resets it)
  int dyn;                 // MODE 0: 1 = dynamic chunk schedule (ctr), 0 = static (chunks g, g + grid, ...)
  // screen (KDT_SCREEN): upper bound u = s~ + eps_a |x||q| + eps_b (sqrt_d |x| + sum|q|)
  float eps_a, eps_b, sqrt_d;
  int full_lists;          // screen: per-lane lists of KT keys (else 4, with a floor; rr_sk.hip KL)
  // MODE 1 (verify, one workgroup per query slot)
  const uint64_t* vin;     // [nlists][slots][KT] screen keys
  int nlists, k_out;
  float* out_scores;       // [b][k_out] (may be null)
  int64_t* out_idx;        // [b][k_out]
  uint64_t* out_keys;      // [slots][KT] exact keys (may be null)
  uint64_t* flag;          // MODE 1: raised (atomic max) to seq when the block needs the exact pass
  int* count;              // MODE 1: [0] blocks flagged so far, [1] blocks verified (slot 0 counts; statistics)
  int seq;                 // this search block's sequence number (> every earlier one)
  int force_incomplete;    // MODE 1 test hook: report the block incomplete
  int wide_verify;         // MODE 1: when the KT candidates cannot prove the top-k, try the wide phase (rescore every
                           // list entry above the largest single-list bound) before raising the flag
  int* wide_count;         // MODE 1: query slots the wide phase proved (statistics; may be null)
  // MODE 0, KT 32, 32 slots, large k (32 < wide_k <= 256): out is [grid][slots][wide_k] — per query the
  // workgroup's top-wide_k of its lane lists — and floors [grid][slots]: no key it dropped is above the floor
  int wide_k;
  uint64_t* floors;
  // MODE 0, KT 32, 32 slots: every key instead of lists, all_keys[q * n + row] for q < b (full-sort path)
  uint64_t* all_keys;
  // int8 screen (KDT_SCREEN8 / 9): corpus = the int8 copy, read as n = ceil(rows8 / 2) kernel rows of two corpus rows
  // each; sx8 / e8 [rows8] the rows' scales and error norms; the block's query pieces p1 at q8 and p2 at q8p2 ([slots][d]
  // each) and their scalars q8s [6][q8s_stride] (launch_q8_stage's layout, offset to the block's first query)
  const int8_t* q8;
  const int8_t* q8p2;
  const float* q8s;
  int q8s_stride;
  const float* sx8;
  const float* e8;
  int64_t rows8;
  int ct8;                 // tiles per chunk of the dynamic schedule (0: the kernel's default)
  int no_guided;           // A/B (RR_SCREEN_GUIDED=0): every chunk CT tiles, no 2-tile chunks at the end
  // Repair mode (the screen's full_lists == 2; rr_sk.hip "Repair"): the screen writes, per chunk and query, the largest
  // upper bound of the chunk's rows (cmax [nchunks][32], order-preserving ords) and zeroes rbits (rbits_words words);
  // the verify (MODE 1, cmax / rbits / nchunks of its block) marks in rbits every chunk whose bound reaches the exact
  // k-th score of a query slot it could not prove (instead of flagging the block) and writes its exact keys to
  // out_keys; repair_count counts those slots. The repair pass (MODE 0 over the fp32 rows) then rescores the listed
  // chunks (rlist, *rcount entries: screen chunk ids, rs = the screen's chunk geometry, rs_rows corpus rows per
  // screen tile) and merge_kernel joins its lists with the verify's keys.
  uint32_t* cmax;
  uint32_t* rbits;
  int rbits_words;
  int cslots;              // MODE 1: query slots of the screen's cmax rows (32, or the bf16 screen's 64)
  int64_t nchunks;
  int* repair_count;
  const int* rlist;
  const int* rcount;
  ChunkGeo rs;
  int rs_rows;
  // MODE 0: the launch's own chunk geometry, computed by launch_sk_args on the host (geo_set = 1): the kernel then
  // starts issuing its first slabs without the ~500 scalar instructions of chunk_geo's 64-bit divisions (r6)
  ChunkGeo geo;
  int geo_set;
};

// Events recorded by the NEXT kernel launch of the calling thread through its launch packet (hipExtLaunchKernelGGL:
// start / stop), instead of hipEventRecord after it: a record is a separate barrier packet that holds the stream's
// next kernel ~3 us on the device (tools/api_cost.hip: kernel -> record -> kernel 4.5 us, kernel with its stop event
// -> kernel 1.4 us, as with nothing between). Taken (and cleared) by launch_sk / launch_sk_args and launch_merge; set
// it right before the launch it is meant for.
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
void set_launch_events(hipEvent_t start, hipEvent_t stop);
LaunchEvents take_launch_events();
#define RR_LAUNCH(K, G, B, SH, S, ...)                                                      \
  do {                                                                                    \
    const ::rr::LaunchEvents le_ = ::rr::take_launch_events();                            \
    if (le_.start || le_.stop)                                                            \
      hipExtLaunchKernelGGL(K, G, B, SH, S, le_.start, le_.stop, 0, __VA_ARGS__);         \
    else                                                                                  \
      hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                    \
  } while (0)

// Split-K streaming kernel (rr_sk.hip): same output contract as launch_fused. sdt = KDT_* (0..3).
// sk_slabs(sdt, d) = 128-byte slabs per wave per row (1..4; bf16 1..2), 0 if d is not supported.
// ring = LDS slab slots per wave (0 = kSkRing): 2. (A third slot ran 5 % slower for fp32 storage and within
// 1 % for bf16 / fp32-split, profiles/r01/kbench_ring.log, and no better from an idle GPU,
// profiles/r02/kbench_transient_ring.log; removed.)
constexpr int kSkRing = 2;
// qslots = query slots per corpus pass (32, or 64 where sk_supports_64: bf16 / fp32-split storage, KT <= 16);
// cand is then [grid][qslots][KT].
int sk_slabs(int sdt, int d);
bool sk_supports_64(int sdt);
size_t sk_lds_bytes(int sdt, bool cos, int ring, int qslots);
hipError_t launch_sk(int sdt, int metric, int kt, int grid, const void* corpus, const float* norms,
                     const float* rscale, const float* queries, int64_t n, int d, int b, uint32_t idx_base,
                     uint64_t* cand, hipStream_t s, int ring = 0, int qslots = 32, uint32_t* ctr = nullptr);
// Any mode: mode 0 (top-KT per workgroup; sdt KDT_SCREEN* = the screens), mode 1 (verify, grid = qslots: KDT_F32_X3
// with 32 slots, or KDT_BF16 — the bf16 screen's verify — with 32 or 64).
hipError_t launch_sk_args(int sdt, int metric, int kt, int mode, int grid, int qslots, const SkArgs& a,
                          hipStream_t s, int ring = 0);

// Merge nlists candidate lists laid out [nlists][slots][in_kt] into the top-kt per query.
// out_keys [slots][kt] (may be null); out_scores/out_idx [b][k_out] (may be null).
// list_stride: elements between consecutive lists (0: slots * in_kt). flag_out: when non-null, raised
// (max) to the largest of the words at in[l * list_stride + slots * in_kt] over the lists — the exchanged
// screened-search flags of every shard. clear_word: when non-null, zeroed (the flag word that follows out_keys in
// an exchange buffer: this search raises no flag, and an earlier one with wider lists may have left a key there).
hipError_t launch_merge(int kt, const uint64_t* in, int nlists, int in_kt, int b, int k_out,
                        uint64_t* out_keys, float* out_scores, int64_t* out_idx, hipStream_t s, int slots = 32,
                        int64_t list_stride = 0, uint64_t* flag_out = nullptr, uint64_t* clear_word = nullptr);

// Top-k selection for 32 < k <= 256 (select_kernel, rr_kernels.hip): grid (32 query slots, parts).
struct SelArgs {
  const uint64_t* in;        // key (list l, query q, pos) at in[l * lstride + q * qstride + pos], pos < kin
  int nlists, kin;
  int64_t lstride, qstride;
  int parts;                 // the lists split into `parts` groups (blockIdx.y); out_keys is [slots][parts][k]
  int sort;                  // 1: output in key order (descending); 0: any order (a stage-1 output)
  const uint64_t* floors;    // list l < nfloors dropped only keys below floors[l * fstride + q] (null: none)
  int nfloors, fstride;
  int64_t xoff;              // >= 0: list l carries a flag word at in[l * lstride + xoff]; their max -> *flag
  int b, k;
  uint64_t* out_keys;        // may be null
  float* out_scores;         // [b][k] (may be null)
  int64_t* out_idx;
  uint64_t* flag;            // floors: raised (atomic max) to seq when a query's top-k is not proven complete
  int* count;                // blocks flagged (statistics; may be null)
  int seq, force_incomplete;
};
hipError_t launch_select(const SelArgs& a, hipStream_t s);

// Repair pass: the set bits of rbits (words words) -> their indices, ascending, in list, and their count in *count.
hipError_t launch_compact_bits(const uint32_t* rbits, int words, int* list, int* count, hipStream_t s);
// Split-K chunk size (tiles) the kernel uses for screen dtype sdt at dimension d (ct8: the int8 screen's setting).
int sk_chunk_tiles(int sdt, int d, int ct8);

// A/B only: a one-workgroup kernel that holds a CU for `us` microseconds (a stand-in for a slower exchange).
hipError_t launch_delay(int us, hipStream_t s);
// Diagnostic: *out = the address of the hardware queue a launch on stream s is dispatched from.
hipError_t launch_queue_probe(uint64_t* out, hipStream_t s);

// Largest |x| of n values (non-negative float bits compared as ints) into *out (device, pre-zeroed).
hipError_t launch_absmax(const float* x, int64_t n, float* out, hipStream_t s);

// Full-score path for k > RR_FUSED_KMAX: keys [b][n] for every (query, doc) pair.
hipError_t launch_full_keys(int kdt, int metric, int grid, const void* corpus, const float* norms,
                            const float* rscale, const float* queries, int64_t n, int d, int b,
                            uint32_t idx_base, uint64_t* keys, hipStream_t s);

// Top-k of b segments of `seg` keys each, sorted descending (rr_topk.hip: radix select, compaction, bitonic tiles,
// rank merges): out [b][k] (row stride k), 0-padded past a segment's non-zero keys. scratch: topk_scratch_bytes(b, k).
size_t topk_scratch_bytes(int b, int64_t k);
hipError_t launch_topk_sorted(const uint64_t* in, int b, int64_t seg, int64_t k, uint64_t* out, void* scratch,
                              hipStream_t s);

// gathered [world][32][k] -> per-query segments [b][world*k].
hipError_t launch_regroup(const uint64_t* gathered, int world, int k, int b, uint64_t* out, hipStream_t s);

// Decode keys [b][k] into scores / indices (-inf / -1 for empty slots).
hipError_t launch_decode(const uint64_t* keys, int b, int k, float* scores, int64_t* idx, hipStream_t s);

// Corpus preparation.
// fp32 (MFMA) and bf16 rows use the pair_unit layout (rr_kernels.hip); conversions take whole rows.
hipError_t launch_permute_f32(const float* in, float* out, int64_t nrows, int d, int inverse, hipStream_t s);
hipError_t launch_f32_to_bf16(const float* in, uint16_t* out, int64_t nrows, int d, hipStream_t s);
// fp32 rows -> f16 (round to nearest even) in the same 8-element pair_unit layout as bf16 storage (the screen copy)
hipError_t launch_f32_to_f16(const float* in, uint16_t* out, int64_t nrows, int d, hipStream_t s);
// fp32 rows (natural order) -> the int8 screen copy: per row sx = max|x| / 127, x8 = clamp(rint(x / sx), +-127),
// e = an upper bound of |x - sx * x8| (rr_kernels.hip f32_to_i8_kernel)
// (bf16 = 1: the rows' bf16 roundings, for bf16 storage's int8 copy)
hipError_t launch_f32_to_i8(const float* in, int64_t nrows, int d, int8_t* out, float* sx, float* e, hipStream_t s,
                            int bf16 = 0);
// The int8 screens' query pieces of a staged batch of b queries (rr_device.h q8_stage_row): q8 = p1 [qc][d] then p2
// [qc][d], q8s [6][qc] (|q|, sum|q|, scale / 64, two-piece residual norm, scale, one-piece residual norm), rows b ..
// 31 (b <= 32) or round_up(b, 64) - 1 zeroed (qc >= that). qcopy (may be null): the fp32 rows are also copied there (fused staging copy).
constexpr int kQ8Scalars = 6;
hipError_t launch_q8_stage(const float* q, int b, int d, int8_t* q8, int qc, float* q8s, float* qcopy, hipStream_t s);
// Load every kernel unit's code object on the current device (rr_create), and the units' own parts of it
hipError_t preload_kernels();
hipError_t preload_sk();
hipError_t preload_topk();
hipError_t launch_row_norms(int dtype, const void* corpus, int64_t n, int d, float* norms, hipStream_t s);
hipError_t launch_synth(int kind, uint64_t seed, int64_t row_begin, int64_t n_rows, int d, float* out,
                        hipStream_t s);
// fp32 rows -> split-f16 storage + |row| (of the fp32 values) + row scales; and back (diagnostics).
hipError_t launch_split_f32(const float* in, int64_t n, int d, void* out, float* norms, float* rscale,
                            hipStream_t s);
hipError_t launch_unsplit_f32(const void* in, const float* rscale, int64_t n, int d, float* out, hipStream_t s);
hipError_t launch_bf16_to_f32(const uint16_t* in, float* out, int64_t nrows, int d, hipStream_t s);

}  // namespace rr
