/*
 * rag_retrieval.h — C-ABI of the MI355X-native dense-retrieval hot path.
 *
 * This library replaces the similarity + top-k core of the reference retrievers
 * (ngray0/RAG-Serving-System, rag_service/core/retriever.py):
 *   - CupyRetriever.__init__          retriever.py:566-592  -> rr_create + rr_load
 *   - CupyRetriever.distance_cosine   retriever.py:594-611  -> fused into rr_search (RR_METRIC_COSINE)
 *   - CupyRetriever.batch_retrieve    retriever.py:686-799  -> rr_search (per-row argpartition/argsort loop
 *                                                              :750-769 becomes one fused top-k)
 *   - SimpleRetriever.retrieve        retriever.py:78-128   -> rr_search (RR_METRIC_DOT, b = 1)
 *   - SimpleRetriever.batch_retrieve  retriever.py:131-166  -> rr_search (RR_METRIC_DOT)
 * The Python side (rag_service_amd.core.retriever) keeps the reference's validation, k-clamping,
 * per-query slicing and document lookup; this ABI only sees validated shapes.
 *
 * Conventions
 *   - Plain pointers and sizes only. Host buffers are caller-owned; device buffers are handle-owned.
 *   - Every int-returning entry point returns RR_OK (0) on success and a negative RR_E* code otherwise;
 *     rr_last_error() then returns a thread-local message.
 *   - One caller thread per handle (the reference calls the retriever from the single BatchProcessor
 *     thread, batch_processor.py:24,95); no internal locking.
 *   - Results are sorted by (score descending, global document index ascending). Slots beyond the
 *     number of documents (k > n) hold score -inf and index -1 (the reference pads with -1,
 *     retriever.py:767-769).
 *   - Scores: RR_METRIC_DOT = fp32 dot product (SimpleRetriever, retriever.py:112);
 *     RR_METRIC_COSINE = clip(dot / (|q|*|d| + 1e-8), -1, 1) in the reference's fp32 operation order
 *     (retriever.py:600-609).
 *   - Sharding: the corpus rows are split into contiguous shards. Shards live either one per process
 *     (rr_init_dist; RCCL communicator from a unique id; per-shard top-k candidates exchanged with one
 *     ncclAllGather over xGMI) or all in one process (rr_create with n_dev > 1; the candidates are
 *     exchanged by peer DMA copies ordered with events; a device may repeat, several shards then
 *     share it). Either way every shard merges the same candidate set on device and ends with the
 *     global result, bit-identical for any shard count.
 */
#ifndef RAG_RETRIEVAL_H
#define RAG_RETRIEVAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RR_ABI_VERSION 9

/* error codes */
#define RR_OK             0
#define RR_E_INVALID     -1   /* bad argument (shape, k, dtype, metric, null pointer) */
#define RR_E_HIP         -2   /* HIP runtime error */
#define RR_E_RCCL        -3   /* RCCL error */
#define RR_E_STATE       -4   /* call out of order (search before load, ...) */
#define RR_E_UNSUPPORTED -5   /* valid request outside what this build implements */
#define RR_E_OOM         -6   /* device allocation failed */
#define RR_E_TIMEOUT     -7   /* device work (an RCCL all-gather waiting for its peers; a stream that never drains)
                                 did not complete within the handle's deadline (rr_set_timeout). The handle is then
                                 FAILED: every later call returns RR_E_STATE; rr_destroy aborts its communicators and
                                 releases nothing else (the process is expected to exit) */

/* corpus storage dtype in HBM (4 bytes per element for both fp32 forms, 2 for bf16) */
#define RR_DTYPE_F32       0  /* fp32 rows stored exactly. Split-K kernel (d % 256 == 0): every corpus and
                                  query value split exactly into three bf16, 6 bf16 MFMAs per product block
                                  (kept partial products exact, dropped terms < 2^-23 |xq|), fp32 accumulate;
                                  register-streaming kernel: v_mfma_f32_32x32x2_f32 (an fp32 fmaf chain).
                                  Either way fp32-class scores (the reference's fp32 GEMM up to summation
                                  order; bit-exact on exactly representable data) */
#define RR_DTYPE_BF16      1  /* bf16 rows (RNE from fp32), bf16 MFMA with fp32 accumulate */
#define RR_DTYPE_F32_SPLIT 2  /* opt-in: fp32 rows stored as f16 hi + lo with a per-row power-of-two scale,
                                  x ~ (hi + lo) * 2^-e with a 22-bit significand (|err| <= 2^-22 |x|); scores
                                  from 3 f16 MFMAs per chunk, fp32 accumulate. Same 4 bytes/element as
                                  RR_DTYPE_F32 but ~1/10 of its matrix-core work (faster; NOT bit-exact fp32) */

/* similarity metric */
#define RR_METRIC_DOT    0    /* SimpleRetriever: raw dot product          (retriever.py:112)      */
#define RR_METRIC_COSINE 1    /* CupyRetriever: clipped cosine similarity  (retriever.py:594-611)  */

/* synthetic corpus kinds for rr_fill_synthetic */
#define RR_SYNTH_EXACT_INT 0  /* x = ((h(seed, row*d+col) mod 255) - 127) * 2^-7 ; exact in bf16 and fp32 */
#define RR_SYNTH_UNIT_NORM 1  /* approx-Gaussian rows (Irwin-Hall of 4 uniforms), L2-normalised in fp32 */

#define RR_UNIQUE_ID_BYTES 128

/* largest k served by the fused single-pass kernel; larger k uses the full-score sort path */
#define RR_FUSED_KMAX 32

typedef struct rr_handle rr_handle;

/* ---- lifecycle ---------------------------------------------------------------------------------- */

/* Create a handle over n_dev local shards on the given devices (HIP ordinals, repeats allowed).
 * devices == NULL means {0}. Loads every kernel unit's code object on each device (tens of ms the first time in a
 * process), so no search pays the runtime's deferred loading.
 * Replaces CupyRetriever.__init__'s device setup (retriever.py:580-586). */
int rr_create(const int* devices, int n_dev, int dtype, int metric, rr_handle** out);

/* Release every device buffer, stream and communicator the handle owns. NULL is a no-op. */
void rr_destroy(rr_handle* h);

/* Thread-local description of the last failure on this thread ("" if none). */
const char* rr_last_error(void);

/* ABI version (RR_ABI_VERSION). */
int rr_abi_version(void);

/* ---- multi-process sharding (one process per GPU) ---------------------------------------------- */

/* Fill out[RR_UNIQUE_ID_BYTES] with an RCCL unique id (call on rank 0, broadcast out-of-band). */
int rr_get_unique_id(char* out);

/* Join a world of `world` processes as `rank`; this process's single local device holds global
 * shard `rank`. Must precede rr_load / rr_load_rows / rr_fill_synthetic. Creates the RCCL communicator
 * for every world size (1 included); every search then exchanges its candidates with ncclAllGather. */
int rr_init_dist(rr_handle* h, int world, int rank, const char* unique_id);

/* Ranks in the handle's RCCL communicator and this process's rank in it (0 and -1 without one). */
int rr_dist_info(const rr_handle* h, int* rccl_ranks, int* rccl_rank);

/* ---- corpus ------------------------------------------------------------------------------------ */

/* Load the whole corpus (row-major fp32, n x d) from host memory. In a multi-process world every
 * rank passes the full matrix and keeps only its shard. Converts to bf16 (RNE) for RR_DTYPE_BF16
 * and precomputes per-row L2 norms for RR_METRIC_COSINE. (retriever.py:576-582)
 * The host array may be pageable; it is streamed through two pinned 32 MiB staging buffers (threaded host
 * copy overlapped with the DMA and the on-device conversion) and is never pinned or modified. */
int rr_load(rr_handle* h, const float* host_corpus, int64_t n, int32_t d);

/* Load only this handle's shard(s): host_rows holds rows [row_begin, row_begin + n_rows) of a
 * corpus of n_total rows. The rows must cover exactly the local shards' ranges. */
int rr_load_rows(rr_handle* h, const float* host_rows, int64_t row_begin, int64_t n_rows,
                 int64_t n_total, int32_t d);

/* Generate a deterministic synthetic corpus of n_total x d directly in HBM (each shard generates its
 * own rows from the global row index, so results do not depend on the shard count). */
int rr_fill_synthetic(rr_handle* h, int kind, uint64_t seed, int64_t n_total, int32_t d);

/* Shape of the loaded corpus and of this handle's local shards. */
int rr_info(const rr_handle* h, int64_t* n_total, int32_t* d, int32_t* n_local_shards,
            int32_t* world_shards);

/* Range [begin, end) of global rows held by local shard `i`. */
int rr_shard_range(const rr_handle* h, int i, int64_t* begin, int64_t* end);

/* Overwrite existing corpus rows in place: host_rows (n_rows x d fp32) replace the rows at the given global indices
 * (each in [0, n_total); a repeated index keeps its last row). Rows outside the local shards are skipped, so every
 * rank of a world may pass the same list. Converted and indexed exactly like loaded rows (storage dtype, per-row
 * norms, the screening copies). Settles and synchronises the handle first. Under rr_init_dist EVERY rank must call it
 * (a collective: the ranks agree by an RCCL min whether the screen's f16 range still holds for every rank's rows).
 * (The reference has no update path: its
 * corpus is replaced by reloading, retriever.py:576-582; rr_load stays that path.) */
int rr_update_rows(rr_handle* h, const float* host_rows, const int64_t* row_idx, int64_t n_rows, int32_t d);

/* Copy rows [row_begin, row_begin + n_rows) of the device-resident corpus back to host as fp32
 * (bf16 corpora are widened). The rows must lie in local shards. Test/diagnostic use. */
int rr_read_rows(const rr_handle* h, int64_t row_begin, int64_t n_rows, float* host_out);

/* The per-row factors the screens read, for rows [row_begin, row_begin + n_rows) of local shards (diagnostic; the GPU
 * tests compare them with NumPy): norms = |x| of the stored values (fp32 sum of squares; cosine, and every screen's
 * bound for either metric), scales / err_norms = the int8 copy's per-row scale max|x| / 127 and rounding-error norm
 * (RR_E_STATE when a shard holding the rows has no int8 copy). Any output may be null. Synchronises the handle. */
int rr_screen_factors(rr_handle* h, int64_t row_begin, int64_t n_rows, float* norms, float* scales,
                      float* err_norms);

/* ---- search ------------------------------------------------------------------------------------ */

/* Synchronous batched search: host queries (b x d fp32, row-major) -> host results
 * out_scores[b*k] (fp32) and out_idx[b*k] (int64 global row index), each row sorted.
 * 1 <= k; k > n is allowed (tail padded with -inf / -1). Replaces batch_retrieve's device part
 * (retriever.py:734-773). */
int rr_search(rr_handle* h, const float* host_q, int32_t b, int32_t d, int32_t k,
              float* out_scores, int64_t* out_idx);

/* Split form of rr_search for serving pipelines and benchmarks:
 *   rr_set_queries   : H2D copy of b x d queries into every local shard's query buffer
 *   rr_search_staged : enqueue the device pipeline on the staged queries (async; results stay in HBM)
 *   rr_synchronize   : wait for all local shard streams
 *   rr_fetch_results : D2H of the last search's results (synchronises first)           */
int rr_set_queries(rr_handle* h, const float* host_q, int32_t b, int32_t d);
int rr_search_staged(rr_handle* h, int32_t k);
int rr_synchronize(rr_handle* h);
int rr_fetch_results(rr_handle* h, float* out_scores, int64_t* out_idx);

/* Shape of the results rr_fetch_results writes: the batch and k of the last search (0, 0 before any
 * search or after a reload). out_scores / out_idx must hold b*k elements. */
int rr_last_shape(const rr_handle* h, int32_t* b, int32_t* k);

/* Pipelined form of rr_search for serving loops: stage the queries through a pinned buffer, enqueue
 * the H2D copy, the search and the D2H copy of its results, and return at once with a ticket. Up to 4
 * searches may be in flight; rr_wait(ticket) blocks until that search's results are on the host and
 * copies them (b*k scores and indices, sorted as rr_search's) into the caller's buffers. Tickets are
 * waited in any order, each exactly once. */
int rr_search_async(rr_handle* h, const float* host_q, int32_t b, int32_t d, int32_t k, int32_t* ticket);
int rr_wait(rr_handle* h, int32_t ticket, float* out_scores, int64_t* out_idx);

/* Queries already on local device 0 (e.g. a torch tensor from the embedding model): device-to-device
 * copy into every local shard's query buffer (skips the reference's .cpu().numpy() round trip,
 * batch_processor.py:92). dev_q is a device pointer on the handle's first local device. */
int rr_set_queries_device(rr_handle* h, const float* dev_q, int32_t b, int32_t d);

/* ---- kernel selection (diagnostics / A-B tests) --------------------------------------------------- */

#define RR_KERNEL_AUTO  0   /* split-K LDS-DMA kernel where the shape allows it (d*elem/8 a multiple of
                               128 bytes, at most 512 bytes; 64 queries per corpus pass for bf16 /
                               fp32-split at k <= 16), else the register-streaming kernel. fp32 storage at
                               k <= 29: the screened search (an f16 screening pass of upper bounds, exact
                               rescoring of the candidates, an exact full pass when the bound cannot prove
                               completeness) — results identical to RR_KERNEL_EXACT; bf16 storage in
                               64-query blocks (33..64 queries) at k <= 13: the screened search over its
                               int8 copy (rr_screen_int8), verified by the bf16 pass's own arithmetic —
                               results identical to RR_KERNEL_EXACT */
#define RR_KERNEL_FUSED 1   /* always the register-streaming kernel (fp32: f32 MFMA) */
#define RR_KERNEL_EXACT 2   /* split-K kernel, every row scored by the storage's exact arithmetic in one pass
                               (no screening) */
#define RR_KERNEL_SCREEN_FALLBACK 3   /* test hook: screened search whose verify always reports the block
                                         incomplete, so the exact fallback pass produces the results */

/* Choose the similarity kernel for k <= RR_FUSED_KMAX searches on this handle. Results of the two kernels
 * differ only by fp32 summation order. */
int rr_set_kernel(rr_handle* h, int kernel);

/* Work schedule of the split-K kernels: 1 (default) = dynamic — each workgroup takes its first chunk of
 * tiles, then the next free one from a device counter, so workgroups on faster CUs take more; 0 = static
 * (chunks dealt round-robin). Results are identical; for A/B measurements. */
int rr_set_schedule(rr_handle* h, int dynamic);

/* Compute streams of the screened search (fp32 and bf16 storage): 2 (default) = consecutive search blocks alternate
 * between two streams, so one block's screen starts while the previous block's screen drains its last chunks
 * and its exact verify runs (the screen then leaves 32 CUs to the verify; verifies that write the same results
 * still follow each other); 1 = every block on one stream, every CU screening; -1 = leave as is. Results are
 * identical. *in_use (may be null): the streams in use (1 or 2). Synchronises the handle's streams when the
 * setting changes. */
int rr_set_compute_streams(rr_handle* h, int32_t n, int32_t* in_use);

/* The screened search's f16 copy (fp32 storage): the screen pass reads an f16 copy of the rows — exactly the
 * values it would round the fp32 rows to in registers — so it streams half the bytes; the verify and every
 * result still come from the fp32 rows (bit-identical results either way). The copy costs 2 bytes per element
 * of HBM and is made at load time when it fits (default). use = 1: keep one (from the next load), 0: free it
 * and screen from the fp32 rows, -1: leave as is. *present (may be null): the copy is in use on every local
 * shard. bf16 storage: the same switch for its int8 copy (rr_screen_int8), *present = that copy on every shard. */
int rr_screen_copy(rr_handle* h, int32_t use, int32_t* present);

/* The screened search's int8 copy (fp32 storage, d a multiple of 512 up to 1024, beside the f16 copy): per row a
 * scale and the rounding error's norm, the rows as int8 — a quarter of the fp32 bytes per screen — against two int8
 * pieces of each query (v_mfma_i32_32x32x32_i8). Its upper bound (exact integer sums + the error norms, Cauchy-
 * Schwarz) is ~8x looser than the f16 copy's, so more rows reach the verify; results are bit-identical either way.
 * Corpora whose blocks re-run switch the handle to repair mode (rr_screen_state), which keeps screening this copy.
 * Made at load time for shards of at least 65536 rows when it fits (default; RR_SCREEN_I8=0 at
 * creation: not made; RR_SCREEN_I8_MIN_ROWS: another row minimum). use = 1: screen it
 * (re-armed; from the next load if none was made), 0: screen the f16 copy, -1: leave as is. *active (may be null):
 * the next search screens the int8 copy on every local shard.
 * bf16 storage: an int8 copy of the bf16 rows (half their bytes), screened against ONE int8 piece per query (32- and
 * 64-query blocks), and verified by the bf16 pass's own arithmetic (DT 9 / DT 1 in rr_sk.hip); it is bf16's only
 * screen (no f16 copy), so use = 0 (or the adaptive pause) leaves bf16 on the exact pass. Made for shards of at least
 * 65536 rows (as above); screened when every row is finite with a norm of at most 2^60 (the bound's arithmetic then
 * stays finite; a larger row leaves the handle on the exact pass). */
int rr_screen_int8(rr_handle* h, int32_t use, int32_t* active);

/* Repair mode (the adaptive screen's answer to corpora whose near-duplicate clusters defeat the screen's lists; see
 * rr_screen_state): query slots, summed over local shards since the corpus was (re)loaded, that the verify could not
 * prove and the in-stream repair pass completed instead — the rows of every chunk whose screen bound reaches the
 * slot's exact k-th score rescored exactly, no host re-run. Synchronises the handle's streams. */
int rr_screen_repairs(rr_handle* h, int64_t* repaired_slots);

/* Screened-search counters since the corpus was (re)loaded: search blocks screened (summed over local
 * shards) and how many of them needed the exact fallback pass. Synchronises the handle's streams. */
int rr_screen_stats(rr_handle* h, int64_t* blocks, int64_t* fallbacks);

/* The same counters plus the exact re-runs the handle actually ran (a staged search whose results are never
 * fetched is superseded by the next one and is not re-run; benchmarks pay flagged - re-runs exact searches
 * themselves) and the query slots whose top-k the verify proved only in its wide phase (every screen-list entry
 * above the largest single-list bound rescored: near-duplicate clusters). Synchronises the handle's streams, which
 * settles the last search. Any pointer may be null. */
int rr_screen_counts(rr_handle* h, int64_t* blocks, int64_t* flagged, int64_t* reruns, int64_t* wide_slots);

/* The screen's adaptive state (fp32 storage): *full_lists = 1 once re-run blocks made the handle switch to REPAIR
 * MODE — the screen keeps full per-lane lists (instead of 4 keys + a floor) and records per chunk of rows the largest
 * bound, and a query slot the verify cannot prove is completed in-stream by rescoring exactly the rows of the chunks
 * whose bound reaches its exact k-th score (rr_screen_repairs), not by a host re-run; *pause_left = search blocks still to run with the
 * one-pass exact kernel because the screen could not prune this corpus; *pauses = how often that happened. Decided
 * from the searches whose results were collected (rr_fetch_results, rr_synchronize, rr_search, rr_wait), whose
 * completeness flag is exchanged between shards: every rank of a world decides identically. Reset at every load.
 * Any pointer may be null. */
int rr_screen_state(rr_handle* h, int32_t* full_lists, int64_t* pause_left, int64_t* pauses);

/* ---- path settings ------------------------------------------------------------------------------------ */

/* Named settings of HOW searches run — never of their results (every path is exact by construction; the GPU tests
 * check each against RR_KERNEL_EXACT). The defaults are the measured best; the options serve measurements and tests
 * that must reach a path on small inputs. Synchronises the handle first. RR_E_INVALID for an unknown name or a value
 * out of range.
 *   screen_grid          screen workgroups at most (default: one per CU)
 *   verify_cus           CUs an overlapping screen leaves to the other compute stream's verify (32)
 *   x_slots              pipelined-exchange buffer sets, 2 or 4 (4)
 *   x_exchange_delay_us  a one-workgroup delay kernel before each exchange's merge, 0..1000 us (0; a stand-in for a
 *                        slower all-gather)
 *   x_host_wait_us       multi-process mode: host wait for a buffer set's previous exchange before a block (500)
 *   x_thread             multi-process mode: issue the exchanges from a second host thread (1; read by rr_init_dist)
 *   wide_verify          the verify's wide phase (1)
 *   screen_ct8           the int8 screen's tiles per chunk: 0 (by shard size), 2 or 4
 *   screen_i8_pieces     fp32 storage's int8 screen: query pieces, 0 (by shard size), 1 or 2
 *   screen_guided        2-tile chunks at the end of a screen launch (1)
 *   screen_full_lists    repair mode from the start and from every load on (0)
 *   screen_i8_min_rows   the int8 copy is made for shards of at least this many rows (65536; the next load)
 *   stage_stream         where a staged batch's copy and int8 pieces are made: 0 the next block's compute stream (0),
 *                        1 / 2 / 3 a staging stream of its own at normal / greatest / least priority (measured slower)
 *   stage_wait_value     a compute stream follows a staging by a stream wait-value packet instead of an event (0) */
int rr_set_option(rr_handle* h, const char* name, int64_t value);
int rr_get_option(const rr_handle* h, const char* name, int64_t* value);

/* "gfx950; product build", or the A/B build's description (RR_AB_ENV: options read from RR_<NAME> environment
 * variables, and RR_AB_NO_VERIFY, which skips the verify and INVALIDATES results — never set by the product Makefile). */
const char* rr_build_info(void);

/* ---- deadline ---------------------------------------------------------------------------------------- */

/* Deadline (milliseconds, 0 = the runtime's unbounded blocking waits) of every host wait on this handle's device
 * work, in both modes: synchronisation, result fetches, rr_wait, query staging, corpus upload / fill and the
 * load-time agreement between ranks. Device work that does not complete in time — an all-gather whose peers never
 * arrive, a stream that never drains — makes the call return RR_E_TIMEOUT naming the rank (multi-process) or the
 * local shard, its device, the stream and the newest search block, and fails the handle. Default 120000; the
 * environment variable RR_TIMEOUT_MS (or its round-3 name RR_DIST_TIMEOUT_MS) overrides it at rr_create.
 * Multi-process mode with the exchange issue thread (x_thread, the default): the caller's wait for that thread to
 * ISSUE its posted exchanges (host work: the all-gather and merge enqueues) is bounded by max(30 s, this deadline),
 * not by a shorter one — the thread's own wake-up can take milliseconds on a loaded host; device work is bounded as
 * above. */
int rr_set_timeout(rr_handle* h, int32_t ms);

/* Diagnostic: the hardware (AQL) queue each of local shard `i`'s five streams dispatches to — out[0] compute
 * stream 0, out[1] compute stream 1, out[2] exchange lane 0, out[3] exchange lane 1, out[4] the staging stream (query
 * copies and the int8 screens' query pieces, at the runtime's least priority) — as queue addresses (equal addresses =
 * one shared in-order queue). Shards on one device share one set of streams. Synchronises the handle. */
int rr_stream_queues(rr_handle* h, int i, uint64_t* out);

/* ---- timing (benchmarks) ----------------------------------------------------------------------- */

/* Enable/disable HIP-event timing of the fused similarity+top-k kernel on local shard 0's stream. */
int rr_set_timing(rr_handle* h, int enable);

/* Sum (ms) and count of timed fused-kernel launches since the last reset; resets when reset != 0. */
int rr_kernel_time(rr_handle* h, double* total_ms, int64_t* launches, int reset);

#ifdef __cplusplus
}
#endif

#endif /* RAG_RETRIEVAL_H */
