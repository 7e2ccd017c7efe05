// rr_api.cpp — C-ABI host side of the MI355X retrieval hot path (see include/rag_retrieval.h).
//
// Owns the device state the reference keeps in CupyRetriever (retriever.py:566-592): the corpus in
// HBM (here row-sharded over devices), plus what the reference recomputes on every call and we keep
// resident: per-row norms (retriever.py:603) and the query/candidate work buffers. One HIP stream per
// local shard; shards exchange their top-k candidates with one RCCL all-gather (new: the reference
// has no collective).
#include "rag_retrieval.h"
#include "rr_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                            \
  do {                                                                                           \
    hipError_t _e = (expr);                                                                      \
    if (_e != hipSuccess)                                                                        \
      return fail(_e == hipErrorOutOfMemory ? RR_E_OOM : RR_E_HIP, "%s failed: %s (%s:%d)", #expr, \
                  hipGetErrorString(_e), __FILE__, __LINE__);                                    \
  } while (0)

#define NCCL_TRY(expr)                                                                       \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess)                                                                   \
      return fail(RR_E_RCCL, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__, \
                  __LINE__);                                                                 \
  } while (0)

constexpr int kXSlots = 4;   // pipelined-exchange buffer sets (Shard::px_keys)
// Staged query buffers (fp32 rows + the int8 screens' pieces), used in turn by consecutive batches: a batch is staged on
// the staging stream while earlier batches are searched, and its buffer's previous readers (four batches back) are
// long done — so the staging never sits in a compute stream's chain (r6; stage_queries)
constexpr int kQBufs = 4;

// Host-side cost of enqueueing (diagnostics: RR_HOST_PROF=1 prints per-call averages at rr_destroy): [0] whole
// rr_search_staged, [1] the pipelined exchange's enqueue, [2] the ncclAllGather call alone, [3] the screened block's
// screen + verify launches; nanoseconds and calls.
struct HostProf {   // (atomics: the exchange issue thread adds to its slots while the caller adds to others)
  std::atomic<int64_t> ns[10] = {}, n[10] = {};
};
inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Shard {
  int dev = 0;
  int cus = 256;
  // Streams (stream, cstream2, xstream, xstream2): one set per DEVICE. Shards on the same device (a test layout of
  // the single-process exchange) share the first one's set (own_streams false): their work serialises on the
  // device anyway, and no stream ever waits on another stream's event across shards of one device (DESIGN §5,
  // "Hardware queues").
  bool own_streams = true;
  hipStream_t stream = nullptr;
  int64_t row_begin = 0, row_end = 0;   // global rows held
  void* corpus = nullptr;                // [rows][d] fp32 or bf16
  uint16_t* scr16 = nullptr;             // fp32 storage: f16 copy of the rows for the screened search (or null)
  // fp32 storage: the int8 screen's copy (rr_sk.hip DT 8; or null): [round_up(rows, 2)][d] int8 rows (a padding row
  // of zeros), per row its scale and error norm ([rows]); per compute stream the queries' int8 pieces and scalars
  int8_t* scr8 = nullptr;
  float* sx8 = nullptr;
  float* e8 = nullptr;
  float* norms = nullptr;                // [round_up(rows, 32) + 32] |row| (pad = 1)
  float* rscale = nullptr;               // [same] split-f16 row scale 2^-e (pad = 1)
  // staged queries, kQBufs buffers used in turn: [q_cap][d] fp32 each (a new batch is copied into one while searches
  // read the others), and — on shards that hold an int8 copy — the int8 screens' pieces of the same rows, [2][q8c][d]
  // (p1, p2) and their scalars [6][q8c] (rr_device.h q8_stage_row; q8c = round_up(q_cap, 64))
  float* qbuf[kQBufs] = {};
  int8_t* q8t[kQBufs] = {};
  float* q8st[kQBufs] = {};
  int q8c = 0;
  // Two compute streams (rr_set_compute_streams): screened blocks of parity 1 run on cstream2 (stream index 1),
  // so block i + 1's screen starts while block i's screen drains its last chunks and its verify runs. Other work
  // runs on `stream` (index 0). Ordering between the two, by events:
  //   ev_q[t][i]  the last screened verify on stream i that read query buffer t: the next staging into buffer t
  //               (staging stream) waits for it; the next verify on the other stream waits for the last one
  //               (they write the same result rows; a pending async D2H of those rows re-records it);
  //   ev_stage[t] buffer t's staging (sstream, below): every stream's first reader of the batch follows it;
  //   ev_fork     `stream` -> cstream2 after other kinds of search; ev_join cstream2 -> `stream` before them.
  hipStream_t cstream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_q[kQBufs][2] = {};
  // with an exchange step the block's keys-ready event (ev_keys) marks the same point of its stream: ev_q is then not
  // recorded, evq_alias points to that event instead (one marker packet fewer in the compute stream per block;
  // ev_keys[x] is re-recorded kXSlots blocks later, on the same stream — a later point, which only orders more)
  hipEvent_t evq_alias[kQBufs][2] = {};
  hipEvent_t evq(int t, int i) const { return evq_alias[t][i] ? evq_alias[t][i] : ev_q[t][i]; }
  // rr_screen_counts (a timed window's close) waits on a record at each stream's tail: a later hipStreamSynchronize or
  // hipDeviceSynchronize (torch.cuda.synchronize) returns at once when a stream's last command is a completed record,
  // but enqueues and awaits a marker of its own, 11-16 us per stream, when it is a kernel or a copy
  // (tools/api_cost.hip "sync_after_done")
  hipEvent_t ev_tail[5] = {};
  bool q_rd[kQBufs][2] = {};   // ev_q[t][i] recorded, no writer of buffer t waited on it yet
  bool fork_pending = false;   // ev_fork was recorded since cstream2 last waited on it
  bool c2_busy = false;        // cstream2 holds work `stream` has not joined
  // Staging (r6): a batch's copy into query buffer t and the int8 screens' pieces of it (ONE fused kernel from a device
  // source) are made once per batch — not per search block, as the r5 prep kernel was — on the compute stream of the
  // next block (stage_stream 0, the default), or on a staging stream of their own (options 1-3: measured slower, every
  // block then follows a cross-stream event). stage_seen[t][i]: compute stream i is ordered after buffer t's
  // latest staging (the other stream follows ev_stage[t]); ns_rd[t]: a search other than a screened block read buffer t
  // on `stream` since its staging (a staging stream's next staging into t waits on ev_fork, recorded after each).
  hipStream_t sstream = nullptr;
  hipEvent_t ev_stage[kQBufs] = {};
  // option stage_wait_value: each staging also writes its sequence number into stage_word[t] (a stream write-value
  // packet after it), and a compute stream follows it by a wait-value packet instead of an event barrier
  uint32_t* stage_word = nullptr;
  uint32_t stage_seq[kQBufs] = {};
  bool stage_seen[kQBufs][2] = {};
  bool ns_rd[kQBufs] = {};
  int last_vsi = -1, last_vq = 0;   // the last screened verify: its stream index and query buffer
  int q_cap = 0;
  uint64_t* cand = nullptr;              // 2 x [grid][64][32] per-workgroup candidates (the screened search
  int cand_grid = 0;                     // alternates the halves by parity; the other paths use half 0)
  int* scount = nullptr;                 // screened search: [0] blocks this shard flagged for the exact pass,
                                         // [1] blocks its verify completed
  int* wcount = nullptr;                 // ... [0] query slots its verify proved in the wide phase, [1] query slots
                                         // the repair pass completed (repair mode)
  // Repair mode (rr_sk.hip "Repair"; observe_settled), per candidate half (block parity): per-chunk maxima of the
  // bound [chunks][32], the verify's chunk marks, their compacted list and its count; made at the first repair-mode
  // block for up to rcap chunks (every chunk geometry of this shard)
  uint32_t* rcmax[2] = {nullptr, nullptr};
  uint32_t* rbits[2] = {nullptr, nullptr};
  int* rlist[2] = {nullptr, nullptr};
  int* rcnt[2] = {nullptr, nullptr};
  int64_t rcap = 0;
  int* pin_scount = nullptr;             // pinned staging of scount / wcount reads (rr_screen_counts) [4], and of
                                         // the result head's flag word at [4] (8 bytes, read_flag)
  uint32_t* ctr = nullptr;               // split-K chunk counters (dynamic schedule), 0 between launches: one per
                                         // compute stream, kCtrStride words apart; then (words 2 and 3 x kCtrStride)
  uint64_t* shard_keys = nullptr;        // [32][k_cap] this shard's top-k (all-gather send buffer)
  uint64_t* gathered = nullptr;          // [world][32][k_cap] (all-gather receive buffer)
  // pipelined exchange (k <= RR_FUSED_KMAX, world > 1): the exchange of search i (all-gather + final
  // merge) runs on xstream while the compute stream already scores search i + 1; buffers alternate by
  // slot (kXSlots of them, in turn: with two compute streams a block's verify ends about a step and a half after its
  // screen began, so a slot is rewritten only after its exchange has had two more steps to finish). px_keys[x] /
  // px_gathered[x] are [64][KMAX] + tail / [world][...].
  hipStream_t xstream = nullptr;
  // Exchanges alternate between two lanes (slot x on lane x & 1): xstream + comm, xstream2 + comm2 (a split of comm),
  // so two exchanges are in flight — each waits for its block's keys on another stream and for its peers, longer
  // than a step on small shards. Their merges write the same result rows: a merge follows the previous one when that
  // ran on the other lane (ev_xdone of last_x).
  hipStream_t xstream2 = nullptr;
  ncclComm_t comm2 = nullptr;
  int last_x = -1;
  uint64_t* px_keys[kXSlots] = {};
  uint64_t* px_gathered[kXSlots] = {};
  hipEvent_t ev_keys[kXSlots] = {};    // compute stream: px_keys[x] written
  hipEvent_t ev_xdone[kXSlots] = {};   // xstream: exchange of slot x finished (buffers free)
  hipEvent_t ev_cdone = nullptr;                // compute stream: a serial (k > KMAX) exchange finished
  // rr_search_async's D2H of the results (local shard 0, on the stream that wrote them last): the next writer of the
  // result rows on another stream — an exchange merge on the other lane, a serial exchange on `stream` — waits for it
  hipEvent_t ev_rcopy = nullptr;
  bool rcopy_pending = false;
  char* out_base = nullptr;              // one allocation: flag word at 0, scores at kOutHead, indices at out_off
  float* out_scores = nullptr;           // [q_cap][k_cap]
  int64_t* out_idx = nullptr;            // [q_cap][k_cap]
  size_t out_off = 0;
  hipEvent_t pin_q_free = nullptr;       // the last H2D out of the handle's pinned query staging completed
  int k_cap = 0;
  // 32 < k <= kWideMax (large k, rr_sk.hip wide output + select_kernel)
  uint64_t* wcand = nullptr;             // [cand_grid][32][kWideMax] per-workgroup top-k lists
  uint64_t* wfloor = nullptr;            // [cand_grid][32] their floors
  uint64_t* wsel = nullptr;              // [32][kSelParts][kWideMax] stage-1 selections
  // full-sort path (k > kWideMax, unsupported shapes, and the exact re-run of an unproven large-k search)
  uint64_t* full_keys = nullptr;         // [32][max(rows, world*k)]
  size_t full_cap = 0;                   // elements
  void* sort_temp = nullptr;
  size_t sort_temp_bytes = 0;
  ncclComm_t comm = nullptr;             // multi-process mode (rr_init_dist)
  hipEvent_t keys_ready = nullptr;       // single-process exchange: shard_keys written
  hipEvent_t copies_done = nullptr;      // single-process exchange: this shard's peer copies issued+done
  std::vector<hipEvent_t> ev;            // timing event pairs (local shard 0 only)
  size_t ev_used = 0;

  int64_t rows() const { return row_end - row_begin; }
};

}  // namespace

// One in-flight rr_search_async batch: a pinned buffer that carries its queries to the device and,
// stream-ordered after the search, its results back.
// A screened block, as its verify sees it: its lists are in candidate half p; results in place (no exchange) or its
// keys + flag word in px_keys[x] (verify_args).
struct VerifyBlock {
  int q0 = 0, bb = 0, k = 0, kt = 0, slots = 0, x = 0, p = 0, seq = 0;
  bool force = false;   // RR_KERNEL_SCREEN_FALLBACK (test hook: report the block incomplete)
};

struct AsyncSlot {
  char* pin = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;   // results landed in pin
  int32_t b = 0, k = 0, ticket = -1;
  bool pending = false;
  bool screened = false;   // the search ran screened blocks, the first with sequence number seq0
  bool narrow = false;     // ... with 16-entry lists where 2k + 2 wanted 32
  bool i8 = false;         // ... screening the int8 copy
  bool full = false, wide = false;   // ... full per-lane lists / the handle's screen_wide at the time
  int blocks = 0;          // ... screened blocks
  int seq0 = 0;
};
constexpr int kAsyncSlots = 4;

namespace {
struct XWorker;
}  // namespace

struct rr_handle {
  int dtype = RR_DTYPE_F32;
  int metric = RR_METRIC_COSINE;
  int32_t d = 0;
  int64_t n_total = 0;
  int world = 1;        // global shard count
  int shard_base = 0;   // global index of local shard 0
  bool dist = false;
  bool loaded = false;
  std::vector<Shard> shards;
  int32_t cur_b = 0;    // last staged batch
  int32_t last_k = 0;   // k of the last search
  int32_t last_b = 0;   // batch of the last search (the shape rr_fetch_results writes)
  bool timing = false;
  int kernel = RR_KERNEL_AUTO;   // rr_set_kernel
  int parity = 0;                // the next search block's parity (candidate half, compute stream)
  XWorker* xw = nullptr;         // multi-process mode: the exchange issue thread (XWorker below; null: inline)
  int xslot = 0;                 // the next pipelined exchange's buffer set (Shard::px_keys)
  double t_ms = 0.0;
  int64_t t_count = 0;
  // pinned host staging for the synchronous search path (rr_set_queries / rr_fetch_results): the queries
  // are copied into pin_q ONCE per batch and every local shard DMAs them from there
  char* pin_out = nullptr;
  size_t pin_out_cap = 0;
  float* pin_q = nullptr;
  size_t pin_q_cap = 0;
  AsyncSlot aslots[kAsyncSlots];
  int32_t next_ticket = 0;
  // screened search (fp32 storage): allowed when every stored |x| < 2^15 (the screen reads x as f16)
  bool screen_ok = false;
  int screen_seq = 0;
  int64_t screen_blocks = 0;
  int64_t screen_reruns = 0;
  bool last_screened = false;   // the last search (rr_search_staged) ran screened blocks
  int last_seq0 = 0;            // ... and its first block's sequence number
  bool last_settled = true;     // ... and its completeness has been checked (settle_screen)
  int last_qpar = 0;            // ... and the query buffer it read
  int qpar = 0;                 // the staged queries live in every shard's qbuf[qpar]
  int dyn_sched = 1;            // split-K kernels: dynamic chunk schedule (rr_set_schedule)
  int streams = 2;              // compute streams for screened blocks (rr_set_compute_streams)
  // (path settings: rr_set_option, kOptions below; results are the same under every value)
  int screen_grid = 1 << 30;    // screen workgroups at most (screen_grid)
  int verify_cus = 32;           // (kVerifyCUs) CUs an overlapping screen leaves to the other stream's verify (verify_cus)
  int xslots = kXSlots;         // pipelined-exchange buffer sets in use (x_slots: 2 or kXSlots)
  int x_delay_us = 0;           // x_exchange_delay_us: a one-workgroup delay kernel on the exchange lane (a stand-in for
                                // a slower all-gather, for measurements and the deadline tests)
  int x_host_wait_us = 500;     // exchange issue thread: host wait for a px slot's previous exchange (x_host_wait_us)
  int x_thread = 1;             // multi-process mode: the exchange issue thread (x_thread; read at rr_init_dist)
  int stage_wv = 0;             // option stage_wait_value (Shard::stage_word)
  int stage_mode = 0;           // where batches are staged (stage_stream): 0 = the next block's compute stream, 1 / 2 / 3 =
                                // a staging stream at normal / greatest / least priority (measured slower: DESIGN §0)
  int screen_copy = 1;          // fp32 storage: keep an f16 copy for the screened search (rr_screen_copy); bf16: the int8 one
  int screen_i8 = 1;            // ... and an int8 copy, screened first (rr_screen_int8; RR_SCREEN_I8=0 at creation: off)
  int ct8 = 0;                  // the int8 screen's tiles per chunk (0: by shard size; screen_ct8)
  int i8_pieces = 0;            // fp32 storage's int8 screen: query pieces, 0 = by shard size (kOnePieceRows), 1 or 2
                                // (screen_i8_pieces)
  int guided = 1;               // split-K chunks: 2-tile chunks at the end of a launch (screen_guided)
  int64_t i8_min_rows = 65536;  // ... for shards of at least this many rows (screen_i8_min_rows, RR_SCREEN_I8_MIN_ROWS): below, a search is
                                // launch-bound and lists holding a large share of the shard's rows leave the looser
                                // bound little to prove with (a 1000-row corpus of real embeddings re-ran blocks)
  bool i8_all = false;          // every shard of the world holds an int8 copy (agreed across ranks at load: finish_all)
  bool last_i8 = false;         // the last search screened the int8 copy
  int64_t narrow_settled = 0;   // settled screened blocks run with 16-entry lists where 2k + 2 wanted 32 (screen_kt)
  int64_t narrow_reruns = 0;    // ... of them re-run exactly
  bool screen_wide = false;     // narrow lists re-ran too often on this corpus: use the wide ones
  bool last_narrow = false;     // the last search ran narrow lists
  bool last_full = false;       // ... full per-lane lists
  bool last_wide = false;       // ... (screen_wide at the time)
  int last_blocks = 0;          // ... this many screened blocks
  bool last_scr_block = false;  // the last block enqueued was a screened one
  // deadline (rr_set_timeout): every host wait on device work polls against it; a miss fails the handle
  int timeout_ms = 120000;
  bool stream_prio = true;      // streams at the runtime's greatest priority (A/B builds: RR_STREAM_PRIORITY=0)
  bool failed = false;
  int wide_verify = 1;          // the verify's wide phase (wide_verify)
  bool host_prof = false;       // RR_HOST_PROF=1 (diagnostics)
  HostProf hp;
  bool ab_no_verify = false;    // A/B builds only (RR_AB_ENV, RR_AB_NO_VERIFY=1): skip the screened search's verify
                                // launch — results invalid; measures what the verify's launch costs the step. The
                                // product library never sets it.
  // adaptive screen (observe_settled): the screen's per-lane lists grow from 4 keys to KT once blocks flag, and
  // screening pauses when even that leaves most blocks to the exact pass — decided from settled searches only
  bool full_lists = false;
  bool full_lists_env = false;              // (screen_full_lists = 1: repair mode from every load on)
  int64_t win_nb = 0, win_nf = 0;           // settled screened blocks of the current window, and re-run ones
  int64_t screen_pause = 0;                 // search blocks still to run without the screen
  int64_t pauses = 0;                       // statistics: pauses so far (since the load)
};

namespace {

// ---- host waits on device work ---------------------------------------------------------------------------------
// Every host wait on the handle's device work is a polled wait against the handle's deadline (rr_set_timeout,
// default 120 s; 0 = the runtime's blocking waits): one process per GPU, an all-gather whose peers never arrive
// would block the caller forever; within one process, a stream that never drains (round 3's one hung run,
// DESIGN §5 "Hardware queues") did. A miss returns RR_E_TIMEOUT naming the rank or shard, the device, the stream
// and the newest search block, and fails the handle (rr_destroy then aborts the communicators and frees nothing
// that queued work may still reference).
template <class Q, class L>
int poll_until(rr_handle* h, Q&& done, L&& label, int scale = 1) {
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t limit_ms = (int64_t)h->timeout_ms * scale;
  for (int i = 0;; ++i) {
    const hipError_t e = done();
    if (e == hipSuccess) return RR_OK;
    if (e != hipErrorNotReady) return fail(RR_E_HIP, "%s failed: %s", label().c_str(), hipGetErrorString(e));
    if ((i & 63) == 63) {   // a short spin first (the common case completes within microseconds), then the clock
      const int64_t ms =
          std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
      if (ms >= limit_ms) {
        (void)hipGetLastError();
        h->failed = true;
        const std::string l = label();
        const char* what = l.c_str();
        if (h->dist)
          return fail(RR_E_TIMEOUT,
                      "rank %d of %d: %s did not complete within %lld ms (newest search block %d); an all-gather is "
                      "probably waiting for a peer rank that never joined",
                      h->shard_base, h->world, what, (long long)limit_ms, h->screen_seq);
        return fail(RR_E_TIMEOUT, "%s did not complete within %lld ms (newest search block %d)", what,
                    (long long)limit_ms, h->screen_seq);
      }
      if (ms >= 2) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else std::this_thread::yield();
    }
  }
}
int failed_handle() {
  return fail(RR_E_STATE, "the handle failed earlier (device work missed its deadline, RR_E_TIMEOUT): destroy it");
}
bool deadline_on(const rr_handle* h) { return h->timeout_ms > 0; }
const char* stream_role(const Shard& s, hipStream_t st) {
  if (st == s.stream) return "compute stream 0";
  if (st == s.cstream2) return "compute stream 1";
  if (st == s.xstream) return "exchange lane 0";
  if (st == s.xstream2) return "exchange lane 1";
  if (st == s.sstream) return "the staging stream";
  return "a work stream";
}
// "shard i (device d), <stream>: <what>" (the rank instead of the shard index in multi-process mode)
std::string wait_label(const rr_handle* h, const Shard& s, const char* stream, const char* what) {
  char buf[256];
  const int i = (int)(&s - h->shards.data());
  snprintf(buf, sizeof buf, "%s %d (device %d), %s: %s", h->dist ? "rank" : "shard", h->dist ? h->shard_base : i,
           s.dev, stream, what);
  return buf;
}
// Stream st waits for event ev — unless ev has already completed, which orders nothing. A cross-stream wait costs HIP a
// barrier packet and ~4.5 us of host time on the next launch of st (tools/api_cost.hip: record + wait + launch 8.7 us
// against 4.1 us for the three calls apart); the query costs 0.08 us. Most of a search block's waits (buffer slots four
// blocks back, the other stream's last staging) are long complete when the block is enqueued.
hipError_t wait_ev(hipStream_t st, hipEvent_t ev) {
  const hipError_t q = hipEventQuery(ev);
  if (q == hipSuccess) return hipSuccess;
  if (q != hipErrorNotReady) return q;
  return hipStreamWaitEvent(st, ev, 0);
}

int xw_drain(rr_handle* h);   // (the exchange issue thread: every posted exchange issued, below)
int wait_stream(rr_handle* h, const Shard& s, hipStream_t st, const char* what = "device work", int scale = 1) {
  if (h->xw)   // every host wait first sees every posted exchange issued
    if (int rc = xw_drain(h)) return rc;
  if (!deadline_on(h)) {
    HIP_TRY(hipStreamSynchronize(st));
    return RR_OK;
  }
  return poll_until(h, [&] { return hipStreamQuery(st); }, [&] { return wait_label(h, s, stream_role(s, st), what); },
                    scale);
}
int wait_event(rr_handle* h, const Shard& s, hipEvent_t ev, const char* what = "device event") {
  if (h->xw)
    if (int rc = xw_drain(h)) return rc;
  if (!deadline_on(h)) {
    HIP_TRY(hipEventSynchronize(ev));
    return RR_OK;
  }
  return poll_until(h, [&] { return hipEventQuery(ev); }, [&] { return wait_label(h, s, "event", what); });
}

int sync_streams(rr_handle* h);   // every local shard's streams idle (defined with the C-ABI's waits)

size_t elem_bytes(int dtype) { return dtype == RR_DTYPE_BF16 ? 2 : 4; }

// Query slots per corpus pass, at most (the split-K kernel serves 64 queries per pass for bf16 and
// fp32-split storage; every other path 32).
constexpr int kMaxSlots = 64;
// Result buffer head (the screened-search flag word, then padding) and the words each exchanged candidate list
// carries after its keys (word 0: the shard's flag).
constexpr size_t kOutHead = 64;
constexpr int kXTail = 8;
// Large k: the split-K kernel's wide output + radix select (no sort of every key) up to this k; the lists of a
// shard are selected in kSelParts groups first when they hold more than 8192 keys per query.
constexpr int kWideMax = 256;
constexpr int kSelParts = 8;
// chunk counters of the two compute streams: one 128-byte line each
constexpr int kCtrStride = 32;

// How each public corpus dtype is stored and multiplied (rr_internal.h KDT_*).
int kdt_of(int dtype) {
  switch (dtype) {
    case RR_DTYPE_BF16: return rr::KDT_BF16;
    case RR_DTYPE_F32_SPLIT: return rr::KDT_F32_SPLIT;
    default: return rr::KDT_F32_MFMA;
  }
}

// Elements of one half of a shard's candidate buffer: [grid][64 slots][32] keys.
size_t cand_half(const Shard& s) { return (size_t)s.cand_grid * kMaxSlots * RR_FUSED_KMAX; }

void shard_range(int64_t n, int world, int g, int64_t* b, int64_t* e) {
  const int64_t per = (n + world - 1) / world;
  *b = std::min<int64_t>(n, (int64_t)g * per);
  *e = std::min<int64_t>(n, *b + per);
}

template <class T>
int dmalloc(T** p, size_t bytes) {
  if (*p) {
    hipFree(*p);
    *p = nullptr;
  }
  if (bytes == 0) bytes = 16;
  HIP_TRY(hipMalloc((void**)p, bytes));
  return RR_OK;
}

int free_shard(Shard& s) {
  hipSetDevice(s.dev);
  for (int t = 0; t < kQBufs; ++t)
    for (void* p : {(void*)s.qbuf[t], (void*)s.q8t[t], (void*)s.q8st[t]})
      if (p) hipFree(p);
  void* ptrs[] = {s.corpus, s.scr16, s.scr8, s.sx8, s.e8, s.norms, s.rscale, s.cand, s.scount, s.ctr, s.stage_word, s.shard_keys, s.gathered, s.out_base,
                  s.full_keys, s.sort_temp, s.wcand, s.wfloor, s.wsel, s.rcmax[0], s.rcmax[1], s.rbits[0], s.rbits[1],
                  s.rlist[0], s.rlist[1], s.rcnt[0], s.rcnt[1]};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (int x = 0; x < kXSlots; ++x) {
    if (s.px_keys[x]) hipFree(s.px_keys[x]);
    if (s.px_gathered[x]) hipFree(s.px_gathered[x]);
    if (s.ev_keys[x]) hipEventDestroy(s.ev_keys[x]);
    if (s.ev_xdone[x]) hipEventDestroy(s.ev_xdone[x]);
  }
  for (hipEvent_t e : s.ev) hipEventDestroy(e);
  s.ev.clear();
  if (s.pin_scount) hipHostFree(s.pin_scount);
  if (s.keys_ready) hipEventDestroy(s.keys_ready);
  if (s.pin_q_free) hipEventDestroy(s.pin_q_free);
  if (s.copies_done) hipEventDestroy(s.copies_done);
  if (s.ev_cdone) hipEventDestroy(s.ev_cdone);
  if (s.ev_rcopy) hipEventDestroy(s.ev_rcopy);
  for (hipEvent_t e : {s.ev_fork, s.ev_join, s.ev_tail[0], s.ev_tail[1], s.ev_tail[2], s.ev_tail[3], s.ev_tail[4]})
    if (e) hipEventDestroy(e);
  for (int t = 0; t < kQBufs; ++t)
    for (hipEvent_t e : {s.ev_stage[t], s.ev_q[t][0], s.ev_q[t][1]})
      if (e) hipEventDestroy(e);
  if (s.comm2) ncclCommDestroy(s.comm2);
  if (s.comm) ncclCommDestroy(s.comm);
  if (s.own_streams)
    for (hipStream_t st : {s.sstream, s.xstream, s.xstream2, s.cstream2, s.stream})
      if (st) hipStreamDestroy(st);
  s = Shard();
  return RR_OK;
}

// Release the shard's int8 screen copy (current device = s.dev; the staged query pieces go with the work buffers).
void free_i8(Shard& s) {
  for (void* p : {(void*)s.scr8, (void*)s.sx8, (void*)s.e8})
    if (p) hipFree(p);
  s.scr8 = nullptr;
  s.sx8 = s.e8 = nullptr;
}

// Allocate the shard's corpus storage for the current range (and norms when cosine).
int alloc_corpus(rr_handle* h, Shard& s) {
  HIP_TRY(hipSetDevice(s.dev));
  const int64_t rows = s.rows();
  if (int rc = dmalloc(&s.corpus, (size_t)std::max<int64_t>(rows, 1) * h->d * elem_bytes(h->dtype))) return rc;
  // the screened search's f16 copy (half the fp32 bytes): only when HBM has room for it — without it the screen
  // reads the fp32 rows and rounds them to f16 in registers (the same values)
  if (s.scr16) HIP_TRY(hipFree(s.scr16));
  s.scr16 = nullptr;
  free_i8(s);
  size_t free_b = 0, total_b = 0;
  const size_t need16 = (size_t)rows * h->d * 2;
  if (h->dtype == RR_DTYPE_F32 && h->screen_copy && rows > 0 && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
      free_b > need16 + (4ull << 30)) {   // leave room for the norms and the search buffers
    if (hipMalloc((void**)&s.scr16, need16) != hipSuccess) {
      s.scr16 = nullptr;
      (void)hipGetLastError();
    }
  }
  // the int8 copy (a quarter of the fp32 bytes; d a multiple of 512 up to 1024), next to the f16 one it falls back to;
  // bf16 storage: the int8 copy of the bf16 rows (half their bytes), its only screen (rr_sk.hip DT 9)
  const bool bf = h->dtype == RR_DTYPE_BF16;
  if ((s.scr16 || (bf && h->screen_copy && rows > 0)) && h->screen_i8 && rows >= h->i8_min_rows &&
      rr::sk_slabs(bf ? rr::KDT_SCREEN9 : rr::KDT_SCREEN8, h->d) && hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    const int64_t r2 = (rows + 1) / 2 * 2;
    const size_t need8 = (size_t)r2 * h->d + 2 * (size_t)r2 * 4;
    if (free_b > need8 + (4ull << 30)) {
      bool ok = hipMalloc((void**)&s.scr8, (size_t)r2 * h->d) == hipSuccess;
      ok = ok && hipMalloc((void**)&s.sx8, (size_t)r2 * 4) == hipSuccess;
      ok = ok && hipMalloc((void**)&s.e8, (size_t)r2 * 4) == hipSuccess;
      // the padding row (odd row counts) is read as the second half of the last kernel row: zeros, scale 0
      if (ok && r2 > rows) {
        ok = hipMemset(s.scr8 + (size_t)rows * h->d, 0, h->d) == hipSuccess;
        ok = ok && hipMemset(s.sx8 + rows, 0, 4) == hipSuccess && hipMemset(s.e8 + rows, 0, 4) == hipSuccess;
      }
      if (!ok) {
        (void)hipGetLastError();
        free_i8(s);
      }
    }
  }
  const int64_t npad = (rows + rr::kTileDocs - 1) / rr::kTileDocs * rr::kTileDocs + rr::kTileDocs;
  if (int rc = dmalloc(&s.norms, (size_t)npad * sizeof(float))) return rc;
  if (int rc = dmalloc(&s.rscale, (size_t)npad * sizeof(float))) return rc;
  // pad with 1.0 so padded rows divide / scale by something finite
  std::vector<float> ones((size_t)npad, 1.0f);
  HIP_TRY(hipMemcpy(s.norms, ones.data(), ones.size() * sizeof(float), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s.rscale, ones.data(), ones.size() * sizeof(float), hipMemcpyHostToDevice));
  return RR_OK;
}

// Whether the handle keeps per-row norms: cosine (the denominator), and every screen's bound for either metric — the
// fp32 screens' eps and the int8 screens' eq |x| and eps terms read |x| (rr_sk.hip epilogue). bf16 storage therefore
// keeps them for dot too (bf16 + dot left them at the 1.0 placeholder, which the int8 bound read).
// Split-f16 rows get theirs (of the fp32 values) during the split.
bool keeps_norms(const rr_handle* h) {
  return h->metric == RR_METRIC_COSINE || h->dtype == RR_DTYPE_F32 || h->dtype == RR_DTYPE_BF16;
}

// bf16 storage's int8 screen: rows of norm at most kBf16ScreenNorm (and queries inside the verify's range check,
// max|q| < 2^15) keep every quantity of the bound finite: |x||q| <= 2^60 2^15 sqrt(d) < 2^81, the estimate and the
// error terms alike, and the cosine denominator. A larger (or overflowing) row norm turns the screen off for the
// handle: the exact pass serves it, which divides by the same fp32 norm.
constexpr float kBf16ScreenNorm = 0x1p60f;

// Per-row norms (keeps_norms) and whether the shard's rows allow the screened search: fp32 storage, every value inside
// the f16 screens' reading (|x| < 2^15); bf16 storage, every int8 error norm finite and every row norm at most
// kBf16ScreenNorm. Returns the shard's verdict in *screen_ok.
int finish_corpus(rr_handle* h, Shard& s, bool* screen_ok) {
  HIP_TRY(hipSetDevice(s.dev));
  const bool f32 = kdt_of(h->dtype) == rr::KDT_F32_MFMA;
  if (keeps_norms(h) && s.rows() > 0 && kdt_of(h->dtype) != rr::KDT_F32_SPLIT)
    HIP_TRY(rr::launch_row_norms(h->dtype == RR_DTYPE_BF16 ? 1 : 0, s.corpus, s.rows(), h->d, s.norms, s.stream));
  *screen_ok = false;
  if (f32) {
    float* dmax = nullptr;
    HIP_TRY(hipMalloc((void**)&dmax, sizeof(float)));
    hipError_t e = hipMemsetAsync(dmax, 0, sizeof(float), s.stream);
    if (e == hipSuccess && s.rows() > 0) e = rr::launch_absmax((const float*)s.corpus, s.rows() * h->d, dmax, s.stream);
    float m = 0.f;
    if (e == hipSuccess) e = hipMemcpyAsync(&m, dmax, sizeof(float), hipMemcpyDeviceToHost, s.stream);
    if (e != hipSuccess) {
      hipFree(dmax);
      return fail(RR_E_HIP, "corpus range check failed: %s", hipGetErrorString(e));
    }
    if (int rc = wait_stream(h, s, s.stream, "the corpus range check")) return rc;
    hipFree(dmax);
    *screen_ok = m < 32768.0f;   // also false for NaN
  } else if (h->dtype == RR_DTYPE_BF16) {
    // the bf16 screen's bound holds for finite rows (every error norm finite: a NaN or infinite value makes its row's
    // NaN or infinite) whose norm keeps its arithmetic finite (kBf16ScreenNorm; an overflowing norm reads +inf)
    *screen_ok = true;
    if (s.scr8 && s.rows() > 0) {
      float* dmax = nullptr;
      HIP_TRY(hipMalloc((void**)&dmax, 2 * sizeof(float)));
      hipError_t e = hipMemsetAsync(dmax, 0, 2 * sizeof(float), s.stream);
      if (e == hipSuccess) e = rr::launch_absmax(s.e8, s.rows(), dmax, s.stream);
      if (e == hipSuccess) e = rr::launch_absmax(s.norms, s.rows(), dmax + 1, s.stream);
      float m[2] = {0.f, 0.f};
      if (e == hipSuccess) e = hipMemcpyAsync(m, dmax, 2 * sizeof(float), hipMemcpyDeviceToHost, s.stream);
      if (e != hipSuccess) {
        hipFree(dmax);
        return fail(RR_E_HIP, "corpus range check failed: %s", hipGetErrorString(e));
      }
      if (int rc = wait_stream(h, s, s.stream, "the corpus range check")) return rc;
      hipFree(dmax);
      *screen_ok = m[0] <= 3.0e38f && m[1] <= kBf16ScreenNorm;   // (false for NaN and infinity)
    }
  }
  return wait_stream(h, s, s.stream, "the corpus norms");
}

// Multi-process mode: every rank's verdicts v[0..n) (0 / 1) reduced to their minimum, element-wise (one RCCL min on
// shard 0's stream), so that data-dependent path choices agree across ranks. `what` names the agreement in errors;
// `scale` multiplies the deadline (ranks reach a load's agreement at different times). Without rr_init_dist: v as is.
int agree_min(rr_handle* h, int* v, int n, const char* what, int scale) {
  if (!h->dist) return RR_OK;
  if (int rc = xw_drain(h)) return rc;   // (its collectives and this one share the communicator)
  Shard& s = h->shards[0];
  HIP_TRY(hipSetDevice(s.dev));
  int* dv = nullptr;
  HIP_TRY(hipMalloc((void**)&dv, (size_t)n * sizeof(int)));
  int rc = RR_OK;
  hipError_t e = hipMemcpyAsync(dv, v, (size_t)n * sizeof(int), hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess) {
    const ncclResult_t r = ncclAllReduce(dv, dv, n, ncclInt32, ncclMin, s.comm, s.stream);
    if (r != ncclSuccess) rc = fail(RR_E_RCCL, "%s failed: %s", what, ncclGetErrorString(r));
  }
  if (e == hipSuccess && rc == RR_OK) rc = wait_stream(h, s, s.stream, what, scale);
  if (e == hipSuccess && rc == RR_OK) e = hipMemcpy(v, dv, (size_t)n * sizeof(int), hipMemcpyDeviceToHost);
  if (!h->failed) hipFree(dv);
  if (rc) return rc;
  if (e != hipSuccess) return fail(RR_E_HIP, "%s failed: %s", what, hipGetErrorString(e));
  return RR_OK;
}

// Finish every local shard; the screened search is allowed only when every shard's range allows it — in a
// multi-process world every rank's shard: the ranks must take the same path, since the screen's list width sizes
// the all-gather and the re-run decisions issue collectives (an RCCL min over the ranks' verdicts). Likewise whether
// EVERY shard holds an int8 copy (each rank allocates its own when its shard is large enough and HBM has room): the
// adaptive screen judges int8-screened searches by their own rule (observe_settled), and ranks must judge alike.
int finish_all(rr_handle* h) {
  bool ok = true, i8 = true;
  for (Shard& s : h->shards) {
    bool sok = false;
    if (int rc = finish_corpus(h, s, &sok)) return rc;
    ok = ok && sok;
    i8 = i8 && (s.scr8 != nullptr || s.rows() == 0);
  }
  int v[2] = {ok ? 1 : 0, i8 ? 1 : 0};
  // ranks finish loading at different times: a generous multiple of the deadline
  if (int rc = agree_min(h, v, 2, "the ranks' screen-range agreement", 10)) return rc;
  h->screen_ok = v[0] != 0;
  h->i8_all = v[1] != 0;
  return RR_OK;
}

// Convert `nr` fp32 rows already on the device (tmp) into the shard's storage at local row `dst_row`.
hipError_t store_rows(rr_handle* h, Shard& s, const float* tmp, int64_t dst_row, int64_t nr) {
  const int d = h->d;
  switch (kdt_of(h->dtype)) {
    case rr::KDT_BF16:
      if (s.scr8)   // the int8 copy of the rows' bf16 roundings
        if (hipError_t e = rr::launch_f32_to_i8(tmp, nr, d, s.scr8 + dst_row * d, s.sx8 + dst_row, s.e8 + dst_row,
                                                s.stream, 1))
          return e;
      return rr::launch_f32_to_bf16(tmp, (uint16_t*)s.corpus + dst_row * d, nr, d, s.stream);
    case rr::KDT_F32_SPLIT:
      return rr::launch_split_f32(tmp, nr, d, (float*)s.corpus + dst_row * d, s.norms + dst_row,
                                  s.rscale + dst_row, s.stream);
    default:
      if (s.scr16)
        if (hipError_t e = rr::launch_f32_to_f16(tmp, s.scr16 + dst_row * d, nr, d, s.stream)) return e;
      if (s.scr8)
        if (hipError_t e = rr::launch_f32_to_i8(tmp, nr, d, s.scr8 + dst_row * d, s.sx8 + dst_row, s.e8 + dst_row,
                                                s.stream))
          return e;
      return rr::launch_permute_f32(tmp, (float*)s.corpus + dst_row * d, nr, d, 0, s.stream);
  }
}

// Host memcpy split over a few threads: one core's memcpy (~10 GB/s) is below PCIe/xGMI DMA rates.
void par_memcpy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kPiece = 4u << 20;
  const int nt = (int)std::min<size_t>(8, (bytes + kPiece - 1) / kPiece);
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  const size_t per = (bytes / nt + 63) & ~(size_t)63;
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; ++t) {
    const size_t o = (size_t)t * per;
    if (o < bytes)
      ts.emplace_back([=] { memcpy((char*)dst + o, (const char*)src + o, std::min(per, bytes - o)); });
  }
  memcpy(dst, src, std::min(per, bytes));
  for (auto& t : ts) t.join();
}

// Copy host fp32 rows into shard storage at local row offset `dst_row` (corpus ingest, main.py:20-23 +
// retriever.py:582). Pipelined over two pinned staging buffers: while chunk c is DMA'd and converted on
// the device (pair_unit permutation, bf16 RNE, or split-f16 + norms + scales), the host copies chunk c + 1
// into the other pinned buffer. The caller's (pageable) array is never pinned or modified.
int upload_rows(rr_handle* h, Shard& s, const float* src, int64_t dst_row, int64_t nrows) {
  HIP_TRY(hipSetDevice(s.dev));
  const int d = h->d;
  const int64_t chunk_rows = std::max<int64_t>(1, (32ll << 20) / ((int64_t)d * 4));
  const size_t chunk_bytes = (size_t)std::min(chunk_rows, nrows) * d * 4;
  float* pin[2] = {nullptr, nullptr};
  float* tmp[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  hipError_t e = hipSuccess;
  for (int i = 0; i < 2 && e == hipSuccess; ++i) {
    e = hipHostMalloc((void**)&pin[i], chunk_bytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&tmp[i], chunk_bytes);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[i], hipEventDisableTiming);
  }
  for (int64_t c = 0, r0 = 0; e == hipSuccess && r0 < nrows; ++c, r0 += chunk_rows) {
    const int i = (int)(c & 1);
    const int64_t nr = std::min(chunk_rows, nrows - r0);
    if (c >= 2) {   // chunk c - 2 has left pin[i] / tmp[i]
      if (int rc = wait_event(h, s, done[i], "a corpus upload chunk")) return rc;   // (a timeout fails the handle)
    }
    par_memcpy(pin[i], src + r0 * d, (size_t)nr * d * 4);
    e = hipMemcpyAsync(tmp[i], pin[i], (size_t)nr * d * 4, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess) e = store_rows(h, s, tmp[i], dst_row + r0, nr);
    if (e == hipSuccess) e = hipEventRecord(done[i], s.stream);
  }
  if (int rc = wait_stream(h, s, s.stream, "the corpus upload")) return rc;   // (a timeout fails the handle)
  for (int i = 0; i < 2; ++i) {
    if (pin[i]) hipHostFree(pin[i]);
    if (tmp[i]) hipFree(tmp[i]);
    if (done[i]) hipEventDestroy(done[i]);
  }
  if (e != hipSuccess)
    return fail(e == hipErrorOutOfMemory ? RR_E_OOM : RR_E_HIP, "corpus upload failed: %s", hipGetErrorString(e));
  return RR_OK;
}

int check_shape(const rr_handle* h, int64_t n, int32_t d) {
  if (n <= 0) return fail(RR_E_INVALID, "corpus must have at least one row (n=%lld)", (long long)n);
  if (n >= 0xFFFFFFFFll) return fail(RR_E_UNSUPPORTED, "n=%lld exceeds the 32-bit index range", (long long)n);
  const int mult = h->dtype == RR_DTYPE_BF16 ? 128 : 64;
  if (d <= 0 || d % mult != 0)
    return fail(RR_E_UNSUPPORTED, "d=%d must be a positive multiple of %d for this dtype", d, mult);
  if (rr::fused_lds_bytes(d, 32, kdt_of(h->dtype)) > 150 * 1024)
    return fail(RR_E_UNSUPPORTED, "d=%d too large for the LDS-resident query image", d);
  return RR_OK;
}

// Work buffers are sized for (q_cap, d, k_cap, rows): a reload (possibly with another d or shard size)
// drops them, and the staged batch / last result shape with them.
int drop_work_buffers(rr_handle* h) {
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    for (hipStream_t st : {s.stream, s.xstream, s.xstream2, s.cstream2, s.sstream})
      if (st)
        if (int rc = wait_stream(h, s, st)) return rc;
    s.c2_busy = s.fork_pending = s.rcopy_pending = false;
    s.last_x = -1;
    for (int t = 0; t < kQBufs; ++t) {
      s.q_rd[t][0] = s.q_rd[t][1] = false;
      s.stage_seen[t][0] = s.stage_seen[t][1] = true;   // (nothing staged: nothing to follow)
      s.ns_rd[t] = false;
      for (void** p : {(void**)&s.qbuf[t], (void**)&s.q8t[t], (void**)&s.q8st[t]}) {
        if (*p) HIP_TRY(hipFree(*p));
        *p = nullptr;
      }
    }
    s.q8c = 0;
    s.last_vsi = -1;
    void** ptrs[] = {(void**)&s.cand, (void**)&s.scount, (void**)&s.ctr, (void**)&s.stage_word, (void**)&s.shard_keys,
                     (void**)&s.gathered,
                     (void**)&s.out_base, (void**)&s.full_keys, &s.sort_temp,
                     (void**)&s.wcand, (void**)&s.wfloor, (void**)&s.wsel, (void**)&s.rcmax[0], (void**)&s.rcmax[1],
                     (void**)&s.rbits[0], (void**)&s.rbits[1], (void**)&s.rlist[0], (void**)&s.rlist[1],
                     (void**)&s.rcnt[0], (void**)&s.rcnt[1]};
    for (void** p : ptrs) {
      if (*p) HIP_TRY(hipFree(*p));
      *p = nullptr;
    }
    for (int x = 0; x < kXSlots; ++x)
      for (uint64_t** p : {&s.px_keys[x], &s.px_gathered[x]}) {
        if (*p) HIP_TRY(hipFree(*p));
        *p = nullptr;
      }
    s.wcount = nullptr;   // (inside scount's allocation, freed above)
    s.q_cap = s.k_cap = s.cand_grid = 0;
    s.rcap = 0;
    s.full_cap = s.sort_temp_bytes = 0;
    s.out_scores = nullptr;
    s.out_idx = nullptr;
    s.out_off = 0;
  }
  h->cur_b = 0;
  h->last_k = 0;
  h->last_b = 0;
  h->parity = 0;
  h->xslot = 0;
  h->screen_blocks = 0;   // the flagged-block counters (scount) were freed above
  h->screen_reruns = 0;
  h->narrow_settled = h->narrow_reruns = 0;
  h->screen_wide = false;
  h->full_lists = h->full_lists_env;
  h->win_nb = h->win_nf = 0;
  h->screen_pause = h->pauses = 0;
  h->last_screened = false;
  h->last_settled = true;
  h->qpar = 0;
  h->loaded = false;
  return RR_OK;
}

int prepare_ranges(rr_handle* h, int64_t n, int32_t d) {
  if (int rc = check_shape(h, n, d)) return rc;
  if (int rc = drop_work_buffers(h)) return rc;
  h->n_total = n;
  h->d = d;
  for (size_t i = 0; i < h->shards.size(); ++i) {
    Shard& s = h->shards[i];
    shard_range(n, h->world, h->shard_base + (int)i, &s.row_begin, &s.row_end);
    if (int rc = alloc_corpus(h, s)) return rc;
  }
  return RR_OK;
}

// Work buffers sized for (b queries, k results).
int ensure_buffers(rr_handle* h, int b, int k) {
  // growing the query buffers (zeroed) and the result head (flag word reset) would drop the last checked search's
  // queries and flag before anyone settled it: settle it first (its exact re-run, if owed, needs both)
  bool grow = false;
  for (const Shard& s : h->shards) grow = grow || b > s.q_cap || k > s.k_cap;
  if (grow && h->last_screened && !h->last_settled)
    if (int rc = rr_synchronize(h)) return rc;
  if (grow)   // no search in flight may still write the buffers about to be replaced
    if (int rc = sync_streams(h)) return rc;
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    if (b > s.q_cap || k > s.k_cap) {
      const int qc = std::max(b, s.q_cap), kc = std::max(k, s.k_cap);
      if (b > s.q_cap) {
        const int rows = (qc + kMaxSlots - 1) / kMaxSlots * kMaxSlots;
        const size_t qb = (size_t)rows * h->d * 4;
        for (int i = 0; i < kQBufs; ++i) {
          if (int rc = dmalloc(&s.qbuf[i], qb)) return rc;
          HIP_TRY(hipMemset(s.qbuf[i], 0, qb));
          // the int8 screens' pieces of the staged rows (shards with an int8 copy): p1, p2 [rows][d] + 6 scalars per row
          if (s.scr8) {
            if (int rc = dmalloc(&s.q8t[i], (size_t)2 * rows * h->d)) return rc;
            if (int rc = dmalloc(&s.q8st[i], (size_t)rr::kQ8Scalars * rows * 4)) return rc;
          }
        }
        s.q8c = s.scr8 ? rows : 0;
        for (int t = 0; t < kQBufs; ++t) s.stage_seen[t][0] = s.stage_seen[t][1] = true;   // (fresh buffers)
      }
      // scores and indices in one allocation, so a search's results come back in ONE D2H copy. The last search's
      // results (and flag word) move to the new allocation: rr_fetch_results after staging a larger batch still
      // returns them.
      char* old = s.out_base;
      const size_t old_off = s.out_off;
      s.out_base = nullptr;
      s.out_off = (kOutHead + (size_t)qc * kc * 4 + 255) & ~(size_t)255;
      if (int rc = dmalloc(&s.out_base, s.out_off + (size_t)qc * kc * 8)) return rc;
      const size_t cnt = (size_t)h->last_b * h->last_k;
      if (old && cnt) {
        HIP_TRY(hipMemcpyAsync(s.out_base, old, kOutHead + cnt * 4, hipMemcpyDeviceToDevice, s.stream));
        HIP_TRY(hipMemcpyAsync(s.out_base + s.out_off, old + old_off, cnt * 8, hipMemcpyDeviceToDevice, s.stream));
        if (int rc = wait_stream(h, s, s.stream)) return rc;
      } else {
        HIP_TRY(hipMemset(s.out_base, 0, kOutHead));   // the screened-search flag word starts at 0
      }
      if (old) HIP_TRY(hipFree(old));
      s.out_scores = (float*)(s.out_base + kOutHead);
      s.out_idx = (int64_t*)(s.out_base + s.out_off);
      // serial exchange lists: [32][k] keys + a flag word (large-k path)
      const size_t per = (size_t)rr::kQSlots * std::max(kc, RR_FUSED_KMAX) + kXTail;
      if (int rc = dmalloc(&s.shard_keys, per * 8)) return rc;
      if (int rc = dmalloc(&s.gathered, (size_t)h->world * per * 8)) return rc;
      HIP_TRY(hipMemset(s.shard_keys, 0, per * 8));
      s.q_cap = qc;
      s.k_cap = kc;
    }
    if (!s.cand) {
      s.cand_grid = s.cus;
      if (int rc = dmalloc(&s.cand, 2 * cand_half(s) * 8)) return rc;
      // scount [2] and wcount [2] in one allocation: rr_screen_counts reads all four in one copy
      if (int rc = dmalloc(&s.scount, 4 * sizeof(int))) return rc;
      HIP_TRY(hipMemset(s.scount, 0, 4 * sizeof(int)));
      s.wcount = s.scount + 2;
      if (!s.pin_scount) HIP_TRY(hipHostMalloc((void**)&s.pin_scount, 8 * sizeof(int), hipHostMallocDefault));
      for (int i = 0; i < 8; ++i) ((volatile int*)s.pin_scount)[i] = 0;
      if (int rc = dmalloc(&s.ctr, 4 * kCtrStride * sizeof(uint32_t))) return rc;
      HIP_TRY(hipMemset(s.ctr, 0, 4 * kCtrStride * sizeof(uint32_t)));
      if (int rc = dmalloc(&s.stage_word, 64)) return rc;
      HIP_TRY(hipMemset(s.stage_word, 0, 64));
      for (int t = 0; t < kQBufs; ++t) s.stage_seq[t] = 0;
    }
    if ((h->world > 1 || h->dist) && !s.px_keys[0]) {
      for (int p = 0; p < kXSlots; ++p) {
        // each exchanged list carries its shard's screened-search flag word after the keys
        const size_t per = (size_t)kMaxSlots * RR_FUSED_KMAX + kXTail;
        if (int rc = dmalloc(&s.px_keys[p], per * 8)) return rc;
        if (int rc = dmalloc(&s.px_gathered[p], (size_t)h->world * per * 8)) return rc;
        HIP_TRY(hipMemset(s.px_keys[p], 0, per * 8));
      }
    }
    if (k > RR_FUSED_KMAX && k <= kWideMax && !s.wcand) {
      if (int rc = dmalloc(&s.wcand, (size_t)s.cand_grid * rr::kQSlots * kWideMax * 8)) return rc;
      if (int rc = dmalloc(&s.wfloor, (size_t)s.cand_grid * rr::kQSlots * 8)) return rc;
      if (int rc = dmalloc(&s.wsel, (size_t)rr::kQSlots * kSelParts * kWideMax * 8)) return rc;
    }
  }
  return RR_OK;
}

// Buffers of the full-key path (every key of the shard, then its top-k sorted: rr_topk.hip), allocated on first use.
int ensure_full_sort(rr_handle* h, Shard& s, int k) {
  const size_t need = (size_t)rr::kQSlots * std::max<int64_t>(s.rows(), (int64_t)h->world * k);
  const size_t tb = rr::topk_scratch_bytes(rr::kQSlots, k);
  if (need > s.full_cap || tb > s.sort_temp_bytes) {
    if (int rc = wait_stream(h, s, s.stream)) return rc;   // the old buffers may still be in use
    if (int rc = wait_stream(h, s, s.cstream2)) return rc;
    s.c2_busy = false;
    if (need > s.full_cap) {
      if (int rc = dmalloc(&s.full_keys, need * 8)) return rc;
      s.full_cap = need;
    }
    if (tb > s.sort_temp_bytes) {
      if (int rc = dmalloc(&s.sort_temp, tb)) return rc;
      s.sort_temp_bytes = tb;
    }
  }
  return RR_OK;
}

// Split-K kernel dtype for a public corpus dtype (rr_sk.hip): exact-split bf16x3 for fp32 storage.
int sk_dtype_of(int dtype) {
  switch (dtype) {
    case RR_DTYPE_BF16: return rr::KDT_BF16;
    case RR_DTYPE_F32_SPLIT: return rr::KDT_F32_SPLIT;
    default: return rr::KDT_F32_X3;
  }
}

// Whether the top-k (k <= RR_FUSED_KMAX) search runs the split-K kernel for this handle.
bool use_sk(const rr_handle* h) {
  if (h->kernel == RR_KERNEL_FUSED) return false;
  return rr::sk_slabs(sk_dtype_of(h->dtype), h->d) != 0;
}

// Screened search (rr_sk.hip "Screened search"): list width for k (>= k + 3 spare, 2k + 2 when it fits),
// 0 when k is too large for it. Where 2k + 2 would need 32-entry lists but k + 3 fits 16 (k = 8..13: BASELINE
// config 3's k = 10), 16-entry lists are used — the screen's cheaper form (smaller inserts, the dynamic schedule)
// — until they prove too narrow for the data: more than 1 in 32 narrow blocks re-run exactly (over at least 64)
// switches the handle to the wide lists (re-armed at the next load).
int screen_kt(const rr_handle* h, int k) {
  int want = std::max(2 * k + 2, k + 3);
  if (want > 16 && k + 3 <= 16 && !h->screen_wide) want = 16;
  if (want <= RR_FUSED_KMAX) return rr::fused_kt(want);
  return k + 3 <= RR_FUSED_KMAX ? RR_FUSED_KMAX : 0;
}
bool narrow_lists(const rr_handle* h, int k) { return std::max(2 * k + 2, k + 3) > 16 && screen_kt(h, k) == 16; }
// (note the list-width switch: observe_settled)

// Error bound of the screen (rr_sk.hip, DT 6 and DT 7 alike: the same f16 values of x, <= 16 MFMAs per wave partial):
// eps = kScreenEpsA |x||q| + kScreenEpsB (sqrt(d) |x| + sum|q|).
//   f16(x): <= 2^-11 |x| + 2^-25 per element; q - c0 - c1: <= 2^-22 |q| + 2^-24.99;
//   fp32 accumulation, any order, of the screen (<= 16 MFMAs x 17 roundings + 8 per score) and of the exact
//   DT 3 score (48 x 17 + 8, plus its dropped split terms <= 4 x 2^-24 |xq|): <= 1.7e-5 and 4.9e-5 of
//   sum |x_k q_k| <= |x||q|.  Sum: 5.54e-4 |x||q| + 2^-24.9 (sum|x| + sum|q|), sum|x| <= sqrt(d) |x|; with
//   an 8 % margin on each.
constexpr float kScreenEpsA = 6.0e-4f;
constexpr float kScreenEpsB = 4.0e-8f;
// DT 7 (the f16 copy) multiplies the query as ONE f16 piece (half the matrix-core work of the two-piece split, which
// measured 3-5 % faster per search: less power drawn, less clock throttling): q - f16(q) <= 2^-11 |q_k| + 2^-25 per
// element adds <= 2^-11 |x||q| + 2^-25 sqrt(d) |x| (the cross term with the rounding of x is < 2^-22 |x||q|, inside
// the margins; 8 instead of 16 MFMAs per wave partial only shrink the accumulation term).
constexpr float kScreen16EpsA = 1.1e-3f;
constexpr float kScreen16EpsB = 7.5e-8f;
// DT 8 (the int8 copy) bounds its own arithmetic exactly from the per-row error norms and the query residual
// (rr_sk.hip epilogue): eps_a / eps_b carry only the exact DT 3 score's error (4.9e-5 |x||q| + the subnormal term)
constexpr float kScreen8EpsA = 6.0e-5f;
constexpr float kScreen8EpsB = 4.0e-8f;

// The int8 copy screens (shards that hold one) unless turned off (rr_screen_int8, rr_screen_copy). (Round 4 gave it up
// for the f16 copy on corpora where blocks re-ran; since r5 repair mode keeps it screening there: observe_settled.)
bool i8_active(const rr_handle* h) { return h->screen_i8 && h->screen_copy; }

// fp32 storage: 32-slot blocks (the int8, f16-copy or fp32-reading screen, DT 3 verify); bf16 storage: 32- and 64-slot
// blocks over the int8 copy on every shard (DT 9 screen with one query piece, DT 1 verify: the bf16 pass's own
// arithmetic), 16-entry lists at most in 64-slot blocks (r6: the 32-slot blocks too — bf16 at the headline batch ran
// the exact pass before, 104 k q/s against fp32 storage's screened 183 k on the same int8 bytes).
bool screened_bf16(const rr_handle* h, int k, int slots) {
  return h->dtype == RR_DTYPE_BF16 && i8_active(h) && h->i8_all &&
         (slots == rr::kQSlots || (slots == kMaxSlots && screen_kt(h, k) <= 16));
}
bool screened(const rr_handle* h, int k, int slots) {
  return (h->kernel == RR_KERNEL_AUTO || h->kernel == RR_KERNEL_SCREEN_FALLBACK) &&
         ((h->dtype == RR_DTYPE_F32 && slots == rr::kQSlots) || screened_bf16(h, k, slots)) && h->screen_ok &&
         screen_kt(h, k) != 0 && use_sk(h) && (h->screen_pause == 0 || h->kernel == RR_KERNEL_SCREEN_FALLBACK);
}

// Adaptive screen (r4): decided from SETTLED searches only — a search whose completeness the host checked when it
// collected the results (settle_screen: rr_fetch_results, rr_synchronize, rr_search; rr_wait). The flag word read
// there is, after an exchange, the largest over every rank's shards, so every rank of a world observes the same
// outcomes in the same order and takes the same decisions at the same search (the list width and the pause change
// the exchanged list width and which collectives run: ranks must agree). Round 3 read the device's flagged-block
// counts asynchronously instead ("a block or two late", rank-dependent) and therefore disabled the pause and the
// narrow -> wide switch under rr_init_dist. A staged search nobody collects is not observed (its outcome is never
// read; the bench pays its re-run itself).
//   * narrow (16-entry) lists -> 32-entry ones when more than 1 in 32 settled narrow blocks re-ran (over >= 64);
//   * windows of >= 32 settled screened blocks of the current configuration: more than 1 in 32 re-ran -> REPAIR MODE
//     (r5; h->full_lists): the screen keeps full per-lane lists (KT keys) and records, per chunk of rows and query, the
//     largest bound; a query slot the verify cannot prove is then not flagged — its exact k-th score bars the chunks
//     to rescore exactly, in-stream (mark / compact / repair pass / merge: rr_sk.hip "Repair"), so a corpus whose
//     near-duplicate clusters defeat the lists (contiguous clusters fill a few workgroups' lists) costs the screen plus
//     the rows of those chunks instead of a whole exact pass per block (the int8 copy keeps screening);
//   * repair mode, and still more than 1 in 2 re-ran (only the f16-range guard or the test hook flag there): pause
//     screening for 1024 blocks (the one-pass exact kernel alone), then probe again. Not while this k screens with the
//     narrow lists (the 32-entry ones are tried first).
// A block counts as re-run when its search was (a flagged search re-runs all its blocks). Reset at every load.
void observe_settled(rr_handle* h, int blocks, bool narrow, bool full, bool wide, bool i8, bool rerun) {
  if (blocks <= 0) return;
  const int nre = rerun ? blocks : 0;
  if (narrow && !h->screen_wide) {
    h->narrow_settled += blocks;
    h->narrow_reruns += nre;
    if (h->narrow_settled >= 64 && h->narrow_reruns * 32 > h->narrow_settled) {
      h->screen_wide = true;   // the wide lists are judged afresh
      h->win_nb = h->win_nf = 0;
      return;
    }
  }
  // a search enqueued under another configuration than the current one (before a switch or a pause) tells nothing
  if (h->screen_pause > 0 || full != h->full_lists || (narrow && h->screen_wide) || wide != h->screen_wide ||
      i8 != i8_active(h))
    return;
  h->win_nb += blocks;
  h->win_nf += nre;
  if (h->win_nb < 32) return;
  if (!h->full_lists) {
    if (h->win_nf * 32 > h->win_nb) {
      h->full_lists = true;   // repair mode; the narrow lists are judged afresh in it (they no longer re-run)
      h->narrow_settled = h->narrow_reruns = 0;
    }
  } else if (h->win_nf * 2 > h->win_nb && !narrow) {
    h->screen_pause = 1024;
    ++h->pauses;
  }
  h->win_nb = h->win_nf = 0;
}
// After a search of `blocks` blocks run during a pause: count the pause down (a fresh window follows it).
void pause_tick(rr_handle* h, int blocks) {
  if (h->screen_pause <= 0) return;
  h->screen_pause = std::max<int64_t>(0, h->screen_pause - blocks);
  if (h->screen_pause == 0) h->win_nb = h->win_nf = 0;
}

// Large k (32 < k <= kWideMax): split-K kernel with wide per-workgroup lists, radix select, completeness check
// (the exact re-run — RR_KERNEL_EXACT — takes the full-sort path).
bool wide(const rr_handle* h, int k) {
  return k > RR_FUSED_KMAX && k <= kWideMax && use_sk(h) && h->kernel != RR_KERNEL_EXACT;
}

// Searches whose completeness is checked on the device and settled by the host (settle_screen).
bool checked(const rr_handle* h, int k, int slots) { return screened(h, k, slots) || wide(h, k); }

int fused_grid(const Shard& s) {
  const int64_t ntiles = (s.rows() + rr::kTileDocs - 1) / rr::kTileDocs;
  const int64_t want = (ntiles + rr::kWaves - 1) / rr::kWaves;
  return (int)std::max<int64_t>(1, std::min<int64_t>(s.cand_grid, want));
}

int next_event_pair(Shard& s, hipEvent_t* a, hipEvent_t* b) {
  while (s.ev.size() < 2 * (s.ev_used + 1)) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    s.ev.push_back(e);
  }
  *a = s.ev[2 * s.ev_used];
  *b = s.ev[2 * s.ev_used + 1];
  ++s.ev_used;
  return RR_OK;
}

int collect_timing(rr_handle* h) {
  if (h->shards.empty()) return RR_OK;
  Shard& s = h->shards[0];
  for (size_t i = 0; i < s.ev_used; ++i) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, s.ev[2 * i], s.ev[2 * i + 1]));
    h->t_ms += ms;
    h->t_count += 1;
  }
  s.ev_used = 0;
  return RR_OK;
}

// Screened blocks alternate between two compute streams (rr_set_compute_streams 2, the default): block i + 1's screen
// runs into block i's last chunks and verify. The screen then leaves kVerifyCUs CUs to the verify (one workgroup per
// query slot, each needing a whole CU's LDS): it runs at once beside the next screen instead of waiting for CUs.
// Measured against one stream and every CU screening (profiles/r02/ab/ab_screen_grid*.txt): +23-45 % per step at
// 125k-250k rows, +2-5 % at 1M-2M.
constexpr int kVerifyCUs = 32;
constexpr int64_t kOnePieceRows = 400000;   // fp32 storage's int8 screen: one query piece from this shard size on,
constexpr int64_t kOnePieceMaxRows = 4000000;   // ... below this one (10M rows, k = 10: no faster, and a block flagged
                                                // in the 20-step window, profiles/r05/final/shard_sweep.jsonl)
bool two_streams(const rr_handle* h, const Shard&) { return h->streams == 2; }
// Screen workgroups on shard s; `alone`: no screened block is in flight on the other stream (its last verify has
// completed: a single search, or the first of a burst), so nothing overlaps this one and every CU screens.
int screen_grid(const rr_handle* h, const Shard& s, bool alone) {
  int g = s.cand_grid;
  if (two_streams(h, s) && !alone) g = std::max(g / 2, g - h->verify_cus);
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min(g, h->screen_grid), (s.rows() + 31) / 32));
}
// Stream index of a screened block of parity p, and a stream by index.
int block_si(const rr_handle* h, const Shard& s, int p) { return p == 1 && two_streams(h, s) ? 1 : 0; }
hipStream_t stream_of(const Shard& s, int si) { return si ? s.cstream2 : s.stream; }
hipStream_t cstream(const rr_handle* h, const Shard& s, int p) { return stream_of(s, block_si(h, s, p)); }
// `stream` follows everything enqueued on cstream2 so far (current device = s.dev).
int join_main(Shard& s) {
  if (!s.c2_busy) return RR_OK;
  HIP_TRY(hipEventRecord(s.ev_join, s.cstream2));
  HIP_TRY(wait_ev(s.stream, s.ev_join));
  s.c2_busy = false;
  for (int t = 0; t < kQBufs; ++t) s.stage_seen[t][0] = s.stage_seen[t][0] || s.stage_seen[t][1];
  return RR_OK;
}
// Work just enqueued on `stream` (another kind of search) that the next cstream2 block follows.
int fork_point(Shard& s) {
  HIP_TRY(hipEventRecord(s.ev_fork, s.stream));
  s.fork_pending = true;
  return RR_OK;
}
int fork_all(rr_handle* h) {
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    if (int rc = fork_point(s)) return rc;
  }
  return RR_OK;
}
// cstream2 follows `stream`'s last fork point (current device = s.dev)
int follow_fork(Shard& s) {
  if (!s.fork_pending) return RR_OK;
  HIP_TRY(wait_ev(s.cstream2, s.ev_fork));
  s.fork_pending = false;
  for (int t = 0; t < kQBufs; ++t) s.stage_seen[t][1] = s.stage_seen[t][1] || s.stage_seen[t][0];
  return RR_OK;
}
// Compute stream si follows the staging of query buffer t (the copy and the int8 pieces, on the staging stream) before
// its first kernel that reads them: one barrier packet per stream and staging, already satisfied when the staging ran
// beside earlier searches.
hipError_t follow_stage(const rr_handle* h, Shard& s, int t, int si) {
  if (s.stage_seen[t][si]) return hipSuccess;
  s.stage_seen[t][si] = true;
  if (h->stage_wv && s.stage_word)   // (uint32 sequence: wraps after 2^32 stagings of one buffer)
    return hipStreamWaitValue32(stream_of(s, si), s.stage_word + t, s.stage_seq[t], hipStreamWaitValueGte, 0xFFFFFFFFu);
  return wait_ev(stream_of(s, si), s.ev_stage[t]);
}

// Stage a batch of queries into every shard's query buffer t, on the staging stream: from pinned host memory (src_dev <
// 0) or device memory on src_dev; then (shards with an int8 copy) the int8 screens' pieces of the batch — the device copy
// fused into the same kernel when the source is on the shard's own device. The buffer's previous readers (kQBufs
// batches back: screened verifies on either compute stream, other kinds of search on `stream`) are waited for on the
// staging stream. pin_ev: record each shard's pin_q_free after its copy.
int stage_queries(rr_handle* h, int t, const void* src, int b, int src_dev, bool pin_ev) {
  const size_t bytes = (size_t)b * h->d * 4;
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    // where: the staging stream, or (stage_stream 0) the compute stream of the next block, in its chain
    const int x = h->stage_mode == 0 ? block_si(h, s, h->parity) : -1;
    const hipStream_t ss = x >= 0 ? stream_of(s, x) : s.sstream;
    if (x == 1) {   // cstream2 after other kinds of search on `stream` (they read query buffers too)
      if (int rc = follow_fork(s)) return rc;
      s.c2_busy = true;
    }
    for (int i = 0; i < 2; ++i) {
      if (s.q_rd[t][i] && i != x) HIP_TRY(wait_ev(ss, s.evq(t, i)));
      s.q_rd[t][i] = false;
    }
    if (s.ns_rd[t] && x < 0) HIP_TRY(wait_ev(ss, s.ev_fork));   // (recorded after every such search)
    s.ns_rd[t] = false;
    const bool pieces = s.q8t[t] && s.scr8 && s.rows() > 0;
    if (src_dev < 0) {
      HIP_TRY(hipMemcpyAsync(s.qbuf[t], src, bytes, hipMemcpyHostToDevice, ss));
    } else if (s.dev == src_dev) {
      if (!pieces) HIP_TRY(hipMemcpyAsync(s.qbuf[t], src, bytes, hipMemcpyDeviceToDevice, ss));
    } else {
      HIP_TRY(hipMemcpyPeerAsync(s.qbuf[t], s.dev, src, src_dev, bytes, ss));
    }
    if (pin_ev) HIP_TRY(hipEventRecord(s.pin_q_free, ss));
    if (pieces) {   // (from the caller's device buffer directly, copying it on the way, when it is on this device)
      const bool fused = src_dev >= 0 && s.dev == src_dev;
      rr::set_launch_events(nullptr, s.ev_stage[t]);   // (ev_stage on the launch packet: no separate record)
      HIP_TRY(rr::launch_q8_stage(fused ? (const float*)src : s.qbuf[t], b, h->d, s.q8t[t], s.q8c, s.q8st[t],
                                  fused ? s.qbuf[t] : nullptr, ss));
    } else {
      HIP_TRY(hipEventRecord(s.ev_stage[t], ss));
    }
    if (h->stage_wv && s.stage_word) HIP_TRY(hipStreamWriteValue32(ss, s.stage_word + t, ++s.stage_seq[t], 0));
    s.stage_seen[t][0] = s.stage_seen[t][1] = false;
    if (x >= 0) s.stage_seen[t][x] = true;
  }
  return RR_OK;
}

// Single-process exchange (several local shards, possibly on the same device): every shard copies every
// other shard's [32][kk] keys into its `gathered` slot with peer DMA, ordered by events. The same
// layout the RCCL all-gather produces in multi-process mode.
int local_gather(rr_handle* h, size_t per) {
  const size_t bytes = per * 8;
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    HIP_TRY(hipEventRecord(s.keys_ready, s.stream));
  }
  for (Shard& dst : h->shards) {
    HIP_TRY(hipSetDevice(dst.dev));
    for (size_t i = 0; i < h->shards.size(); ++i) {
      const Shard& src = h->shards[i];
      if (&src != &dst) HIP_TRY(wait_ev(dst.stream, src.keys_ready));
      HIP_TRY(hipMemcpyPeerAsync(dst.gathered + i * per, dst.dev, src.shard_keys, src.dev, bytes,
                                 dst.stream));
    }
    HIP_TRY(hipEventRecord(dst.copies_done, dst.stream));
  }
  return RR_OK;
}

// Exchange issue thread (multi-process mode, r5). On the 8-GPU shard the caller's thread set the step: ~40 us of host
// enqueue per block against ~34 us of device work (tools/host_calls.py), ~18 us of it the exchange — the all-gather
// call, the merge launch, two event records and two waits on pending events, each ~3.6 us (tools/api_cost.hip). The
// caller now records the block's keys-ready event and posts the exchange; this thread issues it (issue_exchange, in
// post order: the communicators' collectives keep one order on every rank). The caller never runs ahead of it by more
// than x_lag blocks (px_keys slot reuse, enqueue_block), and drains it (every posted exchange issued) before any host
// wait, any collective of its own and any read of the exchange state (last_x, rcopy): a drained worker is idle, so
// the two threads never touch that state or a communicator at the same time. (r4 measured an issue thread 2-6 %
// slower while the device set the step; RR_X_THREAD=0: inline.)
struct XJob {
  int x, q0, bb, k, kt, slots;
};
struct XWorker {
  static constexpr int kRing = 16;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int64_t> posted{0}, done{0};
  std::atomic<bool> stop{false}, sleeping{false};
  std::condition_variable done_cv;      // the caller's wait for issued exchanges, past its short spin (xw_wait)
  std::atomic<bool> waiter{false};
  std::atomic<int> err{0};
  std::string errmsg;   // written by the worker before err (release), read by the caller after it (acquire)
  XJob ring[kRing];
};
// Posted exchanges not yet issued, at most, when a block is enqueued: block i rewrites the px slot of block i - xslots,
// whose exchange must be issued (its ev_xdone recorded) before block i waits on it — so at most xslots - 1 may be
// pending; xslots - 2 keeps one block of slack (2 with the default 4 sets, 0 with RR_X_SLOTS = 2: ADVICE r5, with 2
// sets and a fixed lag of 2 block i waited on a stale ev_xdone and overwrote keys block i - 2's exchange had not read).
int x_lag(const rr_handle* h);

int issue_exchange(rr_handle* h, int x, int q0, int bb, int k, int kt, int slots, int64_t* ns_gather);

void xw_main(rr_handle* h, XWorker* w) {
  int64_t idle_since = now_ns();
  for (;;) {
    const int64_t d = w->done.load(std::memory_order_relaxed);
    if (d < w->posted.load(std::memory_order_acquire)) {
      const XJob j = w->ring[d % XWorker::kRing];
      if (w->err.load(std::memory_order_relaxed) == 0) {
        int64_t ng = 0;
        const int rc = issue_exchange(h, j.x, j.q0, j.bb, j.k, j.kt, j.slots, h->host_prof ? &ng : nullptr);
        if (ng) {
          h->hp.ns[2] += ng;
          ++h->hp.n[2];
        }
        if (rc) {
          w->errmsg = g_err;   // (this thread's message)
          w->err.store(rc, std::memory_order_release);
        }
      }
      w->done.store(d + 1, std::memory_order_seq_cst);
      if (w->waiter.load(std::memory_order_seq_cst)) {   // the caller blocked in xw_wait (past its short spin)
        std::lock_guard<std::mutex> lk(w->mu);
        w->done_cv.notify_all();
      }
      idle_since = now_ns();
      continue;
    }
    if (w->stop.load(std::memory_order_acquire)) return;
    if (now_ns() - idle_since < 200000) {   // spin 200 us after the last job (the next block's comes within ~40 us)
      std::this_thread::yield();
      continue;
    }
    std::unique_lock<std::mutex> lk(w->mu);
    w->sleeping.store(true, std::memory_order_seq_cst);
    if (w->done.load() == w->posted.load() && !w->stop.load())
      w->cv.wait_for(lk, std::chrono::milliseconds(5));
    w->sleeping.store(false, std::memory_order_relaxed);
    idle_since = now_ns();
  }
}

// the worker's first error, reported on the caller's thread
int xw_check(rr_handle* h) {
  XWorker* w = h->xw;
  if (const int e = w->err.load(std::memory_order_acquire)) return fail(e, "exchange issue thread: %s", w->errmsg.c_str());
  return RR_OK;
}
// wait until at most `lag` posted exchanges are not yet issued. Bounded by 30 s or the handle's deadline if longer —
// not by a short deadline: that bounds device work, and the worker only enqueues (its wake-up alone can take
// milliseconds on a loaded host); an RCCL enqueue that blocks on a dead peer is what the bound is for.
int xw_wait(rr_handle* h, int64_t lag) {
  XWorker* w = h->xw;
  if (!w) return RR_OK;
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t limit_ms = std::max<int64_t>(30000, h->timeout_ms);
  auto pending = [&]() {
    return w->posted.load(std::memory_order_relaxed) - w->done.load(std::memory_order_seq_cst) > lag;
  };
  // a short spin (the worker issues a posted exchange within tens of microseconds), then a blocking wait the worker
  // wakes after each exchange it issues (bounded 1 ms waits: a missed wake-up costs at most that)
  while (pending()) {
    if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {
      std::this_thread::yield();
    } else {
      std::unique_lock<std::mutex> lk(w->mu);
      w->waiter.store(true, std::memory_order_seq_cst);
      if (pending()) w->done_cv.wait_for(lk, std::chrono::milliseconds(1));
      w->waiter.store(false, std::memory_order_relaxed);
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(limit_ms)) {
      h->failed = true;
      return fail(RR_E_TIMEOUT, "rank %d of %d: the exchange issue thread did not issue its posted exchanges within "
                  "%lld ms (an all-gather enqueue blocked: a peer rank that never joined?)", h->shard_base, h->world,
                  (long long)limit_ms);
    }
  }
  return xw_check(h);
}
int xw_drain(rr_handle* h) { return xw_wait(h, 0); }
int x_lag(const rr_handle* h) { return std::max(0, h->xslots - 2); }
int xw_post(rr_handle* h, const XJob& j) {
  XWorker* w = h->xw;
  if (int rc = xw_wait(h, XWorker::kRing - 1)) return rc;
  const int64_t p = w->posted.load(std::memory_order_relaxed);
  w->ring[p % XWorker::kRing] = j;
  w->posted.store(p + 1, std::memory_order_seq_cst);
  if (w->sleeping.load(std::memory_order_seq_cst)) {
    std::lock_guard<std::mutex> lk(w->mu);
    w->cv.notify_one();
  }
  return RR_OK;
}
void xw_start(rr_handle* h) {
  if (h->xw || !h->x_thread) return;
  h->xw = new XWorker();
  h->xw->th = std::thread(xw_main, h, h->xw);
}
void xw_stop(rr_handle* h) {
  XWorker* w = h->xw;
  if (!w) return;
  {
    std::lock_guard<std::mutex> lk(w->mu);
    w->stop.store(true, std::memory_order_release);
    w->cv.notify_one();
  }
  w->th.join();   // (it issues every posted exchange first)
  delete w;
  h->xw = nullptr;
}

// Pipelined exchange (k <= RR_FUSED_KMAX, world > 1) of the search block just scored into px_keys[x]:
// each shard's xstream gathers every shard's [32][kt] list (one RCCL all-gather over xGMI with one
// process per GPU, peer copies within one process) into px_gathered[x] and merges it into the results,
// while the compute stream goes on with the next block. px_keys[x] is rewritten kXSlots blocks later and only
// after ev_xdone[x] of every shard that read it (enqueue_block).
// The stream operations of one exchange, after its ev_keys were recorded.
int issue_exchange(rr_handle* h, int x, int q0, int bb, int k, int kt, int slots, int64_t* ns_gather) {
  const size_t slot = (size_t)slots * kt + kXTail;   // keys + the shard's flag word
  const int lane = x & 1;
  for (Shard& dst : h->shards) {
    HIP_TRY(hipSetDevice(dst.dev));
    const hipStream_t xs = lane ? dst.xstream2 : dst.xstream;
    int64_t tp = ns_gather ? now_ns() : 0;
    auto lap = [&](int slot) {   // (RR_HOST_PROF: per-call host time)
      if (!ns_gather) return;
      const int64_t t = now_ns();
      h->hp.ns[slot] += t - tp;
      ++h->hp.n[slot];
      tp = t;
    };
    if (h->dist) {
      HIP_TRY(wait_ev(xs, dst.ev_keys[x]));
      lap(5);
      const int64_t ta = ns_gather ? now_ns() : 0;
      NCCL_TRY(ncclAllGather(dst.px_keys[x], dst.px_gathered[x], slot, ncclUint64, lane ? dst.comm2 : dst.comm, xs));
      if (ns_gather) *ns_gather += now_ns() - ta;
      tp = ns_gather ? now_ns() : 0;
    } else {
      for (size_t i = 0; i < h->shards.size(); ++i) {
        const Shard& src = h->shards[i];
        HIP_TRY(wait_ev(xs, src.ev_keys[x]));
        HIP_TRY(hipMemcpyPeerAsync(dst.px_gathered[x] + i * slot, dst.dev, src.px_keys[x], src.dev, slot * 8, xs));
      }
    }
    if (h->x_delay_us > 0) HIP_TRY(rr::launch_delay(h->x_delay_us, xs));   // (A/B: a slower exchange)
    if (dst.last_x >= 0 && (dst.last_x & 1) != lane) HIP_TRY(wait_ev(xs, dst.ev_xdone[dst.last_x]));
    lap(5);
    if (dst.rcopy_pending) {   // an asynchronous search's result copy still reads these rows (later merges follow this one)
      HIP_TRY(wait_ev(xs, dst.ev_rcopy));
      dst.rcopy_pending = false;
    }
    rr::set_launch_events(nullptr, dst.ev_xdone[x]);   // (recorded by the merge's launch packet)
    HIP_TRY(rr::launch_merge(kt, dst.px_gathered[x], h->world, kt, bb, k, nullptr, dst.out_scores + (size_t)q0 * k,
                             dst.out_idx + (size_t)q0 * k, xs, slots, (int64_t)slot, (uint64_t*)dst.out_base));
    lap(6);
    dst.last_x = x;
  }
  return RR_OK;
}

// Pipelined exchange of the block just scored into px_keys[x] (k <= RR_FUSED_KMAX, an exchange step): ev_keys[x] on the
// block's compute stream, then the exchange's stream operations.
int enqueue_exchange_px(rr_handle* h, int p, int x, int q0, int bb, int k, int kt, int slots, bool scr) {
  const int64_t tk = h->host_prof ? now_ns() : 0;
  for (Shard& s : h->shards) {   // px_keys[x] is written on the block's compute stream (a screened block: its parity's)
    HIP_TRY(hipSetDevice(s.dev));
    // (a screened block with two compute streams recorded it after its verify already: enqueue_block_body)
    if (!(scr && two_streams(h, s))) HIP_TRY(hipEventRecord(s.ev_keys[x], scr ? cstream(h, s, p) : s.stream));
  }
  if (h->host_prof) {
    h->hp.ns[4] += now_ns() - tk;
    ++h->hp.n[4];
  }
  if (h->xw) return xw_post(h, XJob{x, q0, bb, k, kt, slots});
  int64_t ng = 0;
  const int rc = issue_exchange(h, x, q0, bb, k, kt, slots, h->host_prof ? &ng : nullptr);
  if (ng) {
    h->hp.ns[2] += ng;
    ++h->hp.n[2];
  }
  return rc;
}

// Query slots of one corpus pass for a search of b queries at k.
int block_slots(const rr_handle* h, int b, int k) {
  const int kt = rr::fused_kt(k);
  if (b > rr::kQSlots && kt && kt <= 16 && use_sk(h) && rr::sk_supports_64(sk_dtype_of(h->dtype))) return kMaxSlots;
  return rr::kQSlots;
}

// Kernel arguments common to every split-K launch on this shard.
rr::SkArgs sk_base(const rr_handle* h, const Shard& s, const float* qb, int bb) {
  rr::SkArgs a{};
  a.corpus = (const char*)s.corpus;
  a.norms = s.norms;
  a.rscale = s.rscale;
  a.queries = qb;
  a.n = s.rows();
  a.d = h->d;
  a.b = bb;
  a.idx_base = (uint32_t)s.row_begin;
  a.ctr = s.ctr;
  a.dyn = h->dyn_sched;
  a.no_guided = h->guided ? 0 : 1;
  return a;
}

// The verify's arguments (MODE 1) for screened block v on shard s: its screen's nlists lists in candidate half v.p;
// results in place, or (exchange) this shard's exact keys and the block's flag word in px_keys[v.x] (else the flag is
// the result buffer's head).
void verify_args(const rr_handle* h, const Shard& s, const VerifyBlock& v, int nlists, rr::SkArgs* a) {
  const bool multi = h->world > 1 || h->dist;
  a->vin = s.cand + (size_t)v.p * cand_half(s);
  a->nlists = nlists;
  a->k_out = v.k;
  a->out_scores = multi ? nullptr : s.out_scores + (size_t)v.q0 * v.k;
  a->out_idx = multi ? nullptr : s.out_idx + (size_t)v.q0 * v.k;
  a->out_keys = multi ? s.px_keys[v.x] : nullptr;
  a->flag = multi ? s.px_keys[v.x] + (size_t)v.slots * v.kt : (uint64_t*)s.out_base;
  a->count = s.scount;
  a->force_incomplete = v.force ? 1 : 0;
  a->wide_verify = h->wide_verify;
  a->wide_count = s.wcount;
}

// Repair mode's buffers on shard s for up to `chunks` chunks (allocated once per load: any screen geometry of the shard
// has at most one chunk per 32 rows; current device = s.dev, no repair pass of this shard in flight: the first use).
int ensure_repair(Shard& s, int64_t chunks) {
  if (chunks <= s.rcap) return RR_OK;
  const int64_t cap = std::max<int64_t>(chunks, (s.rows() + 31) / 32 + 8);
  for (int i = 0; i < 2; ++i) {
    if (int rc = dmalloc(&s.rcmax[i], (size_t)cap * kMaxSlots * 4)) return rc;
    if (int rc = dmalloc(&s.rbits[i], (size_t)((cap + 31) / 32) * 4)) return rc;
    if (int rc = dmalloc(&s.rlist[i], (size_t)cap * 4)) return rc;
    if (int rc = dmalloc(&s.rcnt[i], 16)) return rc;
  }
  s.rcap = cap;
  return RR_OK;
}

// Enqueue the device pipeline for query block [q0, q0 + bb) (bb <= slots) on every local shard.
int enqueue_block_body(rr_handle* h, int q0, int bb, int k, int slots) {
  const int d = h->d;
  const bool scr = screened(h, k, slots);
  const bool wk = !scr && wide(h, k);
  const int kt = scr ? screen_kt(h, k) : rr::fused_kt(k);
  const bool multi = h->world > 1 || h->dist;   // an exchange step (RCCL with any world, peer copies)
  const bool local_multi = multi && !h->dist;
  const int p = h->parity;
  const int x = h->xslot;   // pipelined-exchange buffer set of this block
  if (scr || wk) {
    ++h->screen_seq;
    ++h->screen_blocks;
  }
  const int seq = h->screen_seq;
  for (size_t si = 0; si < h->shards.size(); ++si) {
    Shard& s = h->shards[si];
    HIP_TRY(hipSetDevice(s.dev));
    // before shard_keys is rewritten, the other shards' copies of its previous contents must be done
    auto wait_copies = [&]() -> hipError_t {
      if (local_multi)
        for (const Shard& o : h->shards)
          if (&o != &s)
            if (hipError_t e = wait_ev(s.stream, o.copies_done)) return e;
      return hipSuccess;
    };
    // pipelined exchange: px_keys[x] is rewritten only after every exchange that read it has finished
    // (its own all-gather; within one process also the other shards' peer copies of it); -1: every slot
    auto wait_px = [&](int slot, hipStream_t ws) -> hipError_t {
      for (int xs = 0; xs < kXSlots; ++xs)
        if (slot < 0 || xs == slot)
          for (const Shard& o : h->shards)
            if (&o == &s || local_multi)
              if (hipError_t e = wait_ev(ws, o.ev_xdone[xs])) return e;
      return hipSuccess;
    };
    const float* qb = s.qbuf[h->qpar] + (size_t)q0 * d;
    float* osc = s.out_scores + (size_t)q0 * k;
    int64_t* oix = s.out_idx + (size_t)q0 * k;
    const uint32_t base = (uint32_t)s.row_begin;
    const bool timed = h->timing && si == 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (timed)
      if (int rc = next_event_pair(s, &e0, &e1)) return rc;
    if (scr) {
      // screened search, on the compute stream: the screen (upper bounds) into cand[p], then the verify (exact
      // DT 3 scores of the KT candidates; results, or this shard's exact keys for the exchange; raises the
      // block's flag word when the bound cannot prove completeness: settle_screen re-runs then). The verify
      // follows in-stream: a cross-stream hand-off costs ~20-25 us of dispatch latency on MI355X
      // (profiles/r02/steps/), more than the ~17 us verify that running it on the exchange stream overlapped.
      // With an exchange, px_keys[x] is rewritten only after its previous exchange (kXSlots blocks back) is done.
      // (two compute streams: parity 1 on cstream2, after the work of the other stream it must follow)
      const bool two = two_streams(h, s);
      const int bsi = block_si(h, s, p), t = h->qpar;
      const hipStream_t cs = stream_of(s, bsi), vs = cs;
      if (two && bsi == 1) {   // after other kinds of search on `stream`
        if (int rc = follow_fork(s)) return rc;
        s.c2_busy = true;
      }
      HIP_TRY(follow_stage(h, s, t, bsi));   // the batch's rows and int8 pieces (staging stream)
      if (multi) {
        // px_keys[x]'s last reader is the exchange of the block kXSlots back. A stream wait on it is a barrier packet in
        // this compute stream's chain (prep, screen, verify): ~10-16 us of device latency per block even when the
        // exchange finished long before the stream reaches it (tools/api_cost.hip, r5 timelines). When the caller runs
        // ahead of the device (the exchange issue thread), the host waits for it instead, before enqueuing — the
        // compute chain then holds no cross-stream barrier; the device still has kXSlots blocks queued.
        // (a short host wait only: an exchange slower than ~0.5 ms gets the stream wait, and the handle's deadline
        // applies where the caller waits for results)
        if (h->xw && h->x_host_wait_us > 0) {
          const int64_t t_end = now_ns() + (int64_t)h->x_host_wait_us * 1000;
          while (hipEventQuery(s.ev_xdone[x]) == hipErrorNotReady && now_ns() < t_end) std::this_thread::yield();
        }
        HIP_TRY(wait_px(x, cs));
      }
      uint64_t* candp = s.cand + (size_t)p * cand_half(s);
      // the f16 copy holds exactly the values the fp32-reading screen rounds to: half the bytes
      const bool bf = h->dtype == RR_DTYPE_BF16;   // (bf16: the int8 copy, DT 9, 32 or 64 slots; verified by the bf16 pass)
      const bool s16 = !bf && s.scr16 && h->screen_copy && rr::sk_slabs(rr::KDT_SCREEN16, d);
      // the int8 copy: a quarter of the fp32 bytes, a bound ~8x looser (more rows reach the verify's wide phase)
      const bool s8 = bf || (s16 && s.scr8 && i8_active(h));
      // one int8 query piece (DT 9) or two (DT 8): one halves the screen's matrix work for a bound ~2x looser (slack
      // 0.0155 vs 0.0079 on unit-norm rows, tests/test_int8_bound.py), so more query slots need the verify's wide
      // phase — a longer verify, which the step pays on small shards and hides on large ones. Measured
      // (profiles/r05/pieces/, window / steady): 1M +15 % / +6 %, 500k +8 % / +11 %, 1.25M k = 10 +14 % / +7 %, 250k
      // -5 % / +4 %, 125k -12 % / -15 %, 10M k = 10 even: one piece from kOnePieceRows rows on — but not in repair
      // mode, whose repair pass rescores every chunk the bound cannot exclude: on contiguous SQuAD clusters the looser
      // bound marked so many that the screen fell to 0.5x the exact kernel (two pieces: 2.0x; profiles/r05/pieces/)
      const bool one_piece =
          bf || (s8 && (h->i8_pieces == 1 || (h->i8_pieces == 0 && !h->full_lists && s.rows() >= kOnePieceRows &&
                                               s.rows() < kOnePieceMaxRows)));
      const int sdt = one_piece ? rr::KDT_SCREEN9 : s8 ? rr::KDT_SCREEN8 : s16 ? rr::KDT_SCREEN16 : rr::KDT_SCREEN;
      const bool alone = !two || s.last_vsi < 0 || s.last_vsi == bsi ||
                         hipEventQuery(s.evq(s.last_vq, s.last_vsi)) == hipSuccess;
      const int sgrid = screen_grid(h, s, alone);
      const int ct8 = h->ct8 > 0 ? h->ct8 : s.rows() < 500000 ? 2 : 4;   // the int8 screen's tiles per chunk (A/B: RR_SCREEN_CT8)
      // repair mode (rr_sk.hip "Repair"): the screen's chunk geometry, which its per-chunk maxima are indexed by
      const bool rmode = h->full_lists && s.rows() > 0 && !h->ab_no_verify;
      rr::ChunkGeo geo{};
      if (rmode) {
        const int64_t kn = s8 ? (s.rows() + 1) / 2 : s.rows();
        geo = rr::chunk_geo((kn + 31) / 32, rr::sk_chunk_tiles(sdt, d, ct8), sgrid, h->guided != 0);
        if (int rc = ensure_repair(s, geo.C)) return rc;
      }
      const int64_t tl = h->host_prof ? now_ns() : 0;
      // (timed: e0 / e1 ride on the prep's and the screen's launch packets — a separate record would hold the next
      // kernel of this stream ~3 us; rr_internal.h set_launch_events)
      if (timed && s.rows() <= 0) HIP_TRY(hipEventRecord(e0, cs));
      if (s.rows() > 0) {
        rr::SkArgs a = sk_base(h, s, qb, bb);
        a.out = candp;
        a.clear_word = multi ? s.px_keys[x] + (size_t)slots * kt : nullptr;   // the verify of this block may raise it
        a.ctr = s.ctr + (cs == s.stream ? 0 : kCtrStride);
        a.sqrt_d = sqrtf((float)d) * (1.0f + 0x1p-20f);
        a.full_lists = rmode ? 2 : 0;   // (repair mode: full lists + per-chunk maxima)
        if (rmode) {
          a.cmax = s.rcmax[p];
          a.rbits = s.rbits[p];
          a.rbits_words = (int)((geo.C + 31) / 32);
        }
        a.eps_a = s16 ? kScreen16EpsA : kScreenEpsA;
        a.eps_b = s16 ? kScreen16EpsB : kScreenEpsB;
        if (s16) a.corpus = (const char*)s.scr16;
        if (s8) {   // the queries' int8 pieces: made when the batch was staged (stage_queries), rows q0 .. q0 + slots
          a.corpus = (const char*)s.scr8;
          a.n = (s.rows() + 1) / 2;
          a.rows8 = s.rows();
          a.q8 = s.q8t[t] + (size_t)q0 * d;
          a.q8p2 = s.q8t[t] + ((size_t)s.q8c + q0) * d;
          a.q8s = s.q8st[t] + q0;
          a.q8s_stride = s.q8c;
          a.sx8 = s.sx8;
          a.e8 = s.e8;
          a.ct8 = ct8;
          a.eps_a = kScreen8EpsA;
          a.eps_b = kScreen8EpsB;
        }
        const int64_t tsc = h->host_prof ? now_ns() : 0;
        if (timed) rr::set_launch_events(e0, e1);
        HIP_TRY(rr::launch_sk_args(sdt, h->metric, kt, 0, sgrid, slots, a, cs));
        if (h->host_prof) {
          h->hp.ns[9] += now_ns() - tsc;
          ++h->hp.n[9];
        }
      }
      if (timed && s.rows() <= 0) HIP_TRY(hipEventRecord(e1, cs));
      // the verify's completion event (the last kernel of the block on this stream records it through its launch
      // packet): with an exchange the keys-ready event, else ev_q (this verify, the last reader of query buffer t here)
      const hipEvent_t vdone = two ? (multi ? s.ev_keys[x] : s.ev_q[t][bsi]) : nullptr;
      bool vdone_set = false;
      // results written in place (no exchange): this verify follows the previous one when that ran on the other
      // stream (the same rows of the result buffer)
      if (two && !multi && s.last_vsi >= 0 && s.last_vsi != bsi)
        HIP_TRY(wait_ev(vs, s.evq(s.last_vq, s.last_vsi)));
      if (s.rows() > 0 && !h->ab_no_verify) {
        rr::SkArgs v = sk_base(h, s, qb, bb);
        VerifyBlock me;
        me.q0 = q0, me.bb = bb, me.k = k, me.kt = kt, me.slots = slots, me.x = x, me.p = p, me.seq = seq;
        me.force = h->kernel == RR_KERNEL_SCREEN_FALLBACK;
        verify_args(h, s, me, sgrid, &v);
        v.seq = seq;
        // repair mode: the verify's exact keys go after the repair pass's lists in this block's candidate half (past the
        // screen's lists, which the verify reads), slots it cannot prove mark chunks; the repair pass rescores the
        // marked chunks' rows exactly and merge_kernel joins both into the results (or this shard's exchanged keys)
        const size_t half = cand_half(s);
        const size_t roff = ((size_t)slots * sgrid * (kt + 1) + 63) / 64 * 64;
        const size_t lkeys = (size_t)slots * kt;
        const int rgrid = (int)std::min<int64_t>({255, (int64_t)s.cand_grid, (int64_t)((half - roff) / lkeys) - 1});
        uint64_t* rbase = s.cand + (size_t)p * half + roff;
        if (rmode) {
          v.out_keys = rbase + (size_t)rgrid * lkeys;
          v.out_scores = nullptr;
          v.out_idx = nullptr;
          v.cmax = s.rcmax[p];
          v.rbits = s.rbits[p];
          v.nchunks = geo.C;
          v.cslots = slots;
          v.repair_count = s.wcount + 1;
        }
        const int xdt = bf ? rr::KDT_BF16 : rr::KDT_F32_X3;   // the storage's exact arithmetic
        if (vdone && !rmode) {
          rr::set_launch_events(nullptr, vdone);
          vdone_set = true;
        }
        HIP_TRY(rr::launch_sk_args(xdt, h->metric, kt, 1, slots, slots, v, vs));
        if (rmode) {
          HIP_TRY(rr::launch_compact_bits(s.rbits[p], (int)((geo.C + 31) / 32), s.rlist[p], s.rcnt[p], vs));
          rr::SkArgs r = sk_base(h, s, qb, bb);
          r.out = rbase;
          r.rlist = s.rlist[p];
          r.rcount = s.rcnt[p];
          r.rs = geo;
          r.rs_rows = s8 ? 64 : 32;
          HIP_TRY(rr::launch_sk_args(xdt, h->metric, kt, 0, rgrid, slots, r, vs));
          if (vdone) {
            rr::set_launch_events(nullptr, vdone);
            vdone_set = true;
          }
          HIP_TRY(rr::launch_merge(kt, rbase, rgrid + 1, kt, bb, k, multi ? s.px_keys[x] : nullptr,
                                   multi ? nullptr : osc, multi ? nullptr : oix, vs, slots));
        }
      } else if (!h->ab_no_verify) {   // a shard without rows contributes empty lists and no flag
        HIP_TRY(hipMemsetAsync(s.px_keys[x], 0, ((size_t)slots * kt + 1) * 8, vs));
      }
      if (h->host_prof) {
        h->hp.ns[3] += now_ns() - tl;
        ++h->hp.n[3];
      }
      if (two) {   // this verify (the last reader of query buffer t on this stream)
        if (!vdone_set) HIP_TRY(hipEventRecord(vdone, vs));   // (no verify launch: a shard without rows, the A/B knob)
        // with an exchange the keys-ready event (enqueue_exchange_px then records none), ev_q's stand-in
        s.evq_alias[t][bsi] = multi ? s.ev_keys[x] : nullptr;
        s.q_rd[t][bsi] = true;
        s.last_vsi = bsi;
        s.last_vq = t;
      }
    } else if (kt) {
      int grid = fused_grid(s);
      HIP_TRY(wait_px(-1, s.stream));   // no screened verify still reads cand or writes the results
      HIP_TRY(follow_stage(h, s, h->qpar, 0));
      s.ns_rd[h->qpar] = true;
      const bool ev_packet = s.rows() > 0 && use_sk(h);   // (timed: events on the launch packet, as above)
      if (timed && !ev_packet) HIP_TRY(hipEventRecord(e0, s.stream));
      if (s.rows() > 0) {
        if (use_sk(h)) {
          const int sgrid = (int)std::max<int64_t>(1, std::min<int64_t>(s.cand_grid, (s.rows() + 31) / 32));
          if (timed) rr::set_launch_events(e0, e1);
          HIP_TRY(rr::launch_sk(sk_dtype_of(h->dtype), h->metric, kt, sgrid, s.corpus, s.norms, s.rscale, qb,
                                s.rows(), d, bb, base, s.cand, s.stream, 0, slots, h->dyn_sched ? s.ctr : nullptr));
          grid = sgrid;
        } else {
          HIP_TRY(rr::launch_fused(kdt_of(h->dtype), h->metric, kt, grid, s.corpus, s.norms, s.rscale, qb,
                                   s.rows(), d, bb, base, s.cand, s.stream));
        }
      } else {
        HIP_TRY(hipMemsetAsync(s.cand, 0, (size_t)slots * kt * 8, s.stream));
      }
      if (timed && !ev_packet) HIP_TRY(hipEventRecord(e1, s.stream));
      if (!multi) {
        HIP_TRY(rr::launch_merge(kt, s.cand, grid, kt, bb, k, nullptr, osc, oix, s.stream, slots));
      } else {
        HIP_TRY(wait_px(x, s.stream));
        HIP_TRY(rr::launch_merge(kt, s.cand, grid, kt, bb, k, s.px_keys[x], nullptr, nullptr, s.stream, slots, 0,
                                 nullptr, s.px_keys[x] + (size_t)slots * kt));
      }
    } else if (wk) {
      // 32 < k <= kWideMax: the split-K kernel keeps per workgroup and query the top-k of its lane lists
      // (wide output, with a floor above everything it dropped), then a radix select over those lists — one
      // stage, or kSelParts groups then their union — gives the shard's top-k and checks it against the
      // floors: unproven -> the block's flag word (the host re-runs the search with the full sort).
      HIP_TRY(wait_px(-1, s.stream));
      HIP_TRY(wait_copies());
      HIP_TRY(follow_stage(h, s, h->qpar, 0));
      s.ns_rd[h->qpar] = true;
      if (timed) HIP_TRY(hipEventRecord(e0, s.stream));
      uint64_t* flagw = multi ? s.shard_keys + (size_t)rr::kQSlots * k : (uint64_t*)s.out_base;
      // the exchanged flag word sits after this k's keys: clear it (earlier searches with a larger k left keys
      // there); the result head's word (single shard) only grows, by sequence number
      if (multi) HIP_TRY(hipMemsetAsync(flagw, 0, sizeof(uint64_t), s.stream));
      if (s.rows() > 0) {
        const int sgrid = (int)std::max<int64_t>(1, std::min<int64_t>(s.cand_grid, (s.rows() + 31) / 32));
        rr::SkArgs a = sk_base(h, s, qb, bb);
        a.out = s.wcand;
        a.wide_k = k;
        a.floors = s.wfloor;
        a.dyn = 0;
        HIP_TRY(rr::launch_sk_args(sk_dtype_of(h->dtype), h->metric, RR_FUSED_KMAX, 0, sgrid, rr::kQSlots, a,
                                   s.stream));
        if (timed) HIP_TRY(hipEventRecord(e1, s.stream));
        rr::SelArgs sa{};
        sa.b = bb;
        sa.k = k;
        sa.xoff = -1;
        sa.flag = flagw;
        sa.count = s.scount;
        sa.seq = seq;
        sa.force_incomplete = h->kernel == RR_KERNEL_SCREEN_FALLBACK;
        const bool two = (int64_t)sgrid * k > 8192;
        if (two) {   // stage 1: the lists in kSelParts groups, each group's top-k (unsorted)
          rr::SelArgs s1 = sa;
          s1.in = s.wcand;
          s1.nlists = sgrid;
          s1.kin = k;
          s1.lstride = (int64_t)rr::kQSlots * k;
          s1.qstride = k;
          s1.parts = kSelParts;
          s1.out_keys = s.wsel;
          HIP_TRY(rr::launch_select(s1, s.stream));
        }
        sa.in = two ? s.wsel : s.wcand;
        sa.nlists = two ? kSelParts : sgrid;
        sa.kin = k;
        sa.lstride = two ? k : (int64_t)rr::kQSlots * k;
        sa.qstride = two ? (int64_t)kSelParts * k : k;
        sa.parts = 1;
        sa.sort = 1;
        sa.floors = s.wfloor;
        sa.nfloors = sgrid;
        sa.fstride = rr::kQSlots;
        sa.out_keys = multi ? s.shard_keys : nullptr;
        sa.out_scores = multi ? nullptr : osc;
        sa.out_idx = multi ? nullptr : oix;
        HIP_TRY(rr::launch_select(sa, s.stream));
      } else {
        if (timed) HIP_TRY(hipEventRecord(e1, s.stream));
        HIP_TRY(hipMemsetAsync(s.shard_keys, 0, (size_t)rr::kQSlots * k * 8, s.stream));
      }
      if (!multi) {   // results read back on the exchange stream (rr_search_async) come after these
        HIP_TRY(hipEventRecord(s.ev_cdone, s.stream));
        HIP_TRY(wait_ev(s.xstream, s.ev_cdone));
        HIP_TRY(wait_ev(s.xstream2, s.ev_cdone));
      }
    } else {
      // k > RR_FUSED_KMAX: all keys of this shard, their top-k sorted (rr_topk.hip). The exchange
      // is serial on the compute stream, after every pipelined exchange still writing results.
      const int64_t rows = s.rows();
      if (int rc = ensure_full_sort(h, s, k)) return rc;
      if (timed) HIP_TRY(hipEventRecord(e0, s.stream));
      HIP_TRY(wait_px(-1, s.stream));   // no pipelined exchange or screened verify still uses the buffers
      HIP_TRY(wait_copies());
      HIP_TRY(follow_stage(h, s, h->qpar, 0));
      s.ns_rd[h->qpar] = true;
      HIP_TRY(hipMemsetAsync(s.shard_keys, 0, (size_t)rr::kQSlots * k * 8, s.stream));
      if (rows > 0) {
        if (use_sk(h)) {   // the split-K kernel's arithmetic, as every other path of this handle
          const int sgrid = (int)std::max<int64_t>(1, std::min<int64_t>(s.cand_grid, (rows + 31) / 32));
          rr::SkArgs a = sk_base(h, s, qb, bb);
          a.out = s.cand;
          a.all_keys = s.full_keys;
          a.dyn = 0;
          HIP_TRY(rr::launch_sk_args(sk_dtype_of(h->dtype), h->metric, RR_FUSED_KMAX, 0, sgrid, rr::kQSlots, a,
                                     s.stream));
        } else {
          const int grid = fused_grid(s);
          HIP_TRY(rr::launch_full_keys(kdt_of(h->dtype), h->metric, grid, s.corpus, s.norms, s.rscale, qb, rows, d,
                                       bb, base, s.full_keys, s.stream));
        }
        if (timed) HIP_TRY(hipEventRecord(e1, s.stream));
        HIP_TRY(rr::launch_topk_sorted(s.full_keys, bb, rows, k, s.shard_keys, s.sort_temp, s.stream));
      } else if (timed) {
        HIP_TRY(hipEventRecord(e1, s.stream));
      }
      if (!multi) HIP_TRY(rr::launch_decode(s.shard_keys, bb, k, osc, oix, s.stream));
    }
  }
  if (!multi) {
    if (scr) h->parity ^= 1;
    return RR_OK;
  }
  if (kt) {
    const int64_t tx = h->host_prof ? now_ns() : 0;
    if (int rc = enqueue_exchange_px(h, p, x, q0, bb, k, kt, slots, scr)) return rc;
    if (h->host_prof) {
      h->hp.ns[1] += now_ns() - tx;
      ++h->hp.n[1];
    }
    h->parity ^= 1;
    h->xslot = (x + 1) % h->xslots;
    return RR_OK;
  }

  // ---- serial exchange (k > RR_FUSED_KMAX): every shard's [32][k] keys to every shard -----------------
  // (large-k lists carry the shard's flag word after the keys)
  const size_t per = (size_t)rr::kQSlots * k + (wk ? kXTail : 0);
  if (h->dist) {   // one process per GPU: one RCCL all-gather over xGMI
    if (int rc = xw_drain(h)) return rc;   // (the pipelined exchanges' collectives come first, on every rank)
    Shard& s = h->shards[0];
    HIP_TRY(hipSetDevice(s.dev));
    NCCL_TRY(ncclAllGather(s.shard_keys, s.gathered, per, ncclUint64, s.comm, s.stream));
  } else if (int rc = local_gather(h, per)) {
    return rc;
  }
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    float* osc = s.out_scores + (size_t)q0 * k;
    int64_t* oix = s.out_idx + (size_t)q0 * k;
    if (s.rcopy_pending) {   // an asynchronous search's result copy (on an exchange lane) still reads these rows
      HIP_TRY(wait_ev(s.stream, s.ev_rcopy));
      s.rcopy_pending = false;
    }
    if (wk) {   // the world lists' union -> top-k (radix select), and the largest of their flag words
      rr::SelArgs sa{};
      sa.in = s.gathered;
      sa.nlists = h->world;
      sa.kin = k;
      sa.lstride = (int64_t)per;
      sa.qstride = k;
      sa.parts = 1;
      sa.sort = 1;
      sa.xoff = (int64_t)rr::kQSlots * k;
      sa.b = bb;
      sa.k = k;
      sa.flag = (uint64_t*)s.out_base;
      sa.out_scores = osc;
      sa.out_idx = oix;
      HIP_TRY(rr::launch_select(sa, s.stream));
    } else {
      const int64_t seg = (int64_t)h->world * k;
      HIP_TRY(rr::launch_regroup(s.gathered, h->world, k, bb, s.full_keys, s.stream));
      HIP_TRY(rr::launch_topk_sorted(s.full_keys, bb, seg, k, s.shard_keys, s.sort_temp, s.stream));
      HIP_TRY(rr::launch_decode(s.shard_keys, bb, k, osc, oix, s.stream));
    }
    // later pipelined exchanges write the results after this one
    HIP_TRY(hipEventRecord(s.ev_cdone, s.stream));
    HIP_TRY(wait_ev(s.xstream, s.ev_cdone));
    HIP_TRY(wait_ev(s.xstream2, s.ev_cdone));
    s.last_x = -1;
  }
  return RR_OK;
}

// Enqueue one block: a screened block goes on its parity's compute stream; any other block runs on `stream`
// after everything on cstream2, and later cstream2 blocks follow it.
int enqueue_block(rr_handle* h, int q0, int bb, int k, int slots) {
  if (h->xw)   // the exchange of the block xslots back (its px slot's last reader) must be issued
    if (int rc = xw_wait(h, x_lag(h))) return rc;
  const bool scr = screened(h, k, slots);
  if (!scr)
    for (Shard& s : h->shards) {
      HIP_TRY(hipSetDevice(s.dev));
      if (int rc = join_main(s)) return rc;
      s.last_vsi = -1;
    }
  if (int rc = enqueue_block_body(h, q0, bb, k, slots)) return rc;
  h->last_scr_block = scr;
  return scr ? RR_OK : fork_all(h);
}

// A new batch goes into the query buffer the last search did not read: every reader of a query buffer runs on
// the compute stream, where the new batch's copy is ordered after them. The last checked search can be re-run
// only while its buffer is intact, so it is settled first when its buffer is the one about to be rewritten
// (two batches staged, no search).
int begin_stage(rr_handle* h, int* nq) {
  const int t = (h->qpar + 1) % kQBufs;
  if (h->last_screened && !h->last_settled && h->last_qpar == t)
    if (int rc = rr_synchronize(h)) return rc;

  *nq = t;
  return RR_OK;
}

// ---- path settings (rr_set_option) -----------------------------------------------------------------------------
// Every option picks HOW a search runs — grid sizes, list widths, query pieces, the exchange's buffering — never its
// results: each path is exact by construction and the GPU tests check them against the exact kernel. Defaults are the
// measured best; the options exist for measurements and for tests that reach a path on small inputs.
// (Re)create every device's staging stream at the priority of stage_stream mode (1 normal, 2 greatest, 3 least).
int make_stage_streams(rr_handle* h, int mode) {
  int least = 0, greatest = 0;
  HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
  const int prio = mode == 2 ? greatest : mode == 3 ? least : 0;
  for (Shard& s : h->shards) {
    if (!s.own_streams) continue;
    HIP_TRY(hipSetDevice(s.dev));
    if (s.sstream) HIP_TRY(hipStreamDestroy(s.sstream));
    s.sstream = nullptr;
    HIP_TRY(hipStreamCreateWithPriority(&s.sstream, hipStreamNonBlocking, prio));
  }
  for (Shard& s : h->shards)   // shards on one device share the first one's
    for (const Shard& o : h->shards)
      if (o.own_streams && o.dev == s.dev) {
        s.sstream = o.sstream;
        break;
      }
  return RR_OK;
}

struct OptionDesc {
  const char* name;
  int64_t lo, hi;
};
const OptionDesc kOptions[] = {
    {"screen_grid", 1, 1 << 30},        // screen workgroups at most
    {"verify_cus", 0, 256},             // CUs an overlapping screen leaves to the other stream's verify
    {"x_slots", 2, kXSlots},            // pipelined-exchange buffer sets: 2 or 4 (even: each slot stays on one
                                        // compute stream, which ev_keys' use as ev_q's stand-in assumes)
    {"x_exchange_delay_us", 0, 1000},   // a delay kernel on the exchange lane per exchange (a slower all-gather)
    {"x_host_wait_us", 0, 100000},      // exchange issue thread: host wait for a slot's previous exchange
    {"x_thread", 0, 1},                 // multi-process mode: the exchange issue thread (before rr_init_dist)
    {"wide_verify", 0, 1},              // the verify's wide phase
    {"screen_ct8", 0, 8},               // the int8 screen's tiles per chunk (0: by shard size; 2 or 4)
    {"screen_i8_pieces", 0, 2},         // fp32 storage's int8 screen: query pieces (0: by shard size)
    {"screen_guided", 0, 1},            // 2-tile chunks at the end of a screen launch
    {"screen_full_lists", 0, 1},        // repair mode from the start (and from every load on)
    {"screen_i8_min_rows", 0, INT64_MAX / 2},   // the int8 copy for shards of at least this many rows (next load)
    {"stage_stream", 0, 3},             // batches staged on: 0 the next block's compute stream, 1 / 2 / 3 the staging
                                        // stream at normal / greatest / least priority
    {"stage_wait_value", 0, 1},         // a compute stream follows a staging by a stream wait-value packet, not an event
};

int64_t* option_field64(rr_handle* h, const std::string& n) { return n == "screen_i8_min_rows" ? &h->i8_min_rows : nullptr; }
int* option_field(rr_handle* h, const std::string& n) {
  if (n == "screen_grid") return &h->screen_grid;
  if (n == "verify_cus") return &h->verify_cus;
  if (n == "x_slots") return &h->xslots;
  if (n == "x_exchange_delay_us") return &h->x_delay_us;
  if (n == "x_host_wait_us") return &h->x_host_wait_us;
  if (n == "x_thread") return &h->x_thread;
  if (n == "wide_verify") return &h->wide_verify;
  if (n == "screen_ct8") return &h->ct8;
  if (n == "screen_i8_pieces") return &h->i8_pieces;
  if (n == "screen_guided") return &h->guided;
  if (n == "stage_stream") return &h->stage_mode;
  if (n == "stage_wait_value") return &h->stage_wv;
  return nullptr;
}
int set_option(rr_handle* h, const OptionDesc& o, int64_t v) {
  const std::string n = o.name;
  if (v < o.lo || v > o.hi || (n == "x_slots" && v != 2 && v != kXSlots) ||
      (n == "screen_ct8" && v != 0 && v != 2 && v != 4))
    return fail(RR_E_INVALID, "option %s = %lld out of range", o.name, (long long)v);
  if (n == "x_slots") h->xslot = 0;   // (the caller synchronised: no slot in use)
  if (n == "screen_full_lists") {
    h->full_lists_env = v != 0;
    h->full_lists = v != 0;
    h->win_nb = h->win_nf = 0;
    return RR_OK;
  }
  if (n == "stage_stream" && v != h->stage_mode && v > 0) {   // (the caller synchronised: the stream is idle)
    if (int rc = make_stage_streams(h, (int)v)) return rc;
  }
  if (int64_t* f = option_field64(h, n)) *f = v;
  else *option_field(h, n) = (int)v;
  return RR_OK;
}
const OptionDesc* find_option(const char* name) {
  for (const OptionDesc& o : kOptions)
    if (name && strcmp(o.name, name) == 0) return &o;
  return nullptr;
}

}  // namespace

// =================================================================================================
// C-ABI
// =================================================================================================
extern "C" {

const char* rr_last_error(void) { return g_err.c_str(); }

int rr_abi_version(void) { return RR_ABI_VERSION; }

int rr_create(const int* devices, int n_dev, int dtype, int metric, rr_handle** out) {
  g_err.clear();
  if (!out) return fail(RR_E_INVALID, "out is null");
  *out = nullptr;
  if (dtype != RR_DTYPE_F32 && dtype != RR_DTYPE_BF16 && dtype != RR_DTYPE_F32_SPLIT)
    return fail(RR_E_INVALID, "bad dtype %d", dtype);
  if (metric != RR_METRIC_DOT && metric != RR_METRIC_COSINE) return fail(RR_E_INVALID, "bad metric %d", metric);
  int def = 0;
  if (!devices) {
    devices = &def;
    n_dev = 1;
  }
  if (n_dev < 1) return fail(RR_E_INVALID, "n_dev=%d", n_dev);
  int ndev_avail = 0;
  HIP_TRY(hipGetDeviceCount(&ndev_avail));
  rr_handle* h = new rr_handle();
  h->dtype = dtype;
  h->metric = metric;
  h->world = n_dev;
  h->shards.resize(n_dev);
#ifdef RR_AB_ENV
  if (const char* e = getenv("RR_STREAM_PRIORITY")) h->stream_prio = atoi(e) != 0;   // (A/B builds only)
#endif
  for (int i = 0; i < n_dev; ++i) {
    Shard& s = h->shards[i];
    if (devices[i] < 0 || devices[i] >= ndev_avail) {
      for (int j = i; j < n_dev; ++j) h->shards[j].own_streams = false;   // nothing created for them yet
      rr_destroy(h);
      return fail(RR_E_INVALID, "device %d not available (%d devices)", devices[i], ndev_avail);
    }
    s.dev = devices[i];
    hipError_t e = hipSetDevice(s.dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&s.cus, hipDeviceAttributeMultiprocessorCount, s.dev);
    // Streams: one set of four per device, shared by every shard on it (Shard::own_streams), created at the
    // runtime's greatest priority: HIP keeps a separate pool of GPU_MAX_HW_QUEUES hardware queues per priority, so
    // none of ours shares an in-order hardware queue with a normal-priority stream of the process — RCCL's internal
    // streams (whose barrier packets wait for all-gathers), the null stream, torch's (DESIGN §5 "Hardware queues").
    const Shard* owner = nullptr;
    for (int j = 0; j < i; ++j)
      if (h->shards[j].dev == s.dev) {
        owner = &h->shards[j];
        break;
      }
    if (owner) {
      s.own_streams = false;
      s.stream = owner->stream;
      s.cstream2 = owner->cstream2;
      s.xstream = owner->xstream;
      s.xstream2 = owner->xstream2;
      s.sstream = owner->sstream;
    } else {
      int least = 0, greatest = 0;
      if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
      const int prio = h->stream_prio ? greatest : least;
      // creation order = the order the hardware queues are handed out in (least used first)
      for (hipStream_t* st : {&s.stream, &s.xstream, &s.xstream2, &s.cstream2})
        if (e == hipSuccess) e = hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio);
      // (no staging stream by default: stage_stream 0 stages on the compute streams; rr_set_option makes one)
    }
    if (e != hipSuccess) {
      for (int j = i + 1; j < n_dev; ++j) h->shards[j].own_streams = false;
      rr_destroy(h);
      return fail(RR_E_HIP, "device %d setup failed: %s", devices[i], hipGetErrorString(e));
    }
  }
  for (Shard& s : h->shards) {   // every kernel unit loaded on each device now, not inside the first search
    if (!s.own_streams) continue;
    if (hipError_t e = hipSetDevice(s.dev)) {
      rr_destroy(h);
      return fail(RR_E_HIP, "device %d: %s", s.dev, hipGetErrorString(e));
    }
    if (hipError_t e = rr::preload_kernels()) {
      rr_destroy(h);
      return fail(RR_E_HIP, "device %d: loading the kernels failed: %s", s.dev, hipGetErrorString(e));
    }
  }
  for (Shard& s : h->shards) {   // single-process exchange events (unused with one shard)
    hipError_t e = hipSetDevice(s.dev);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.keys_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.copies_done, hipEventDisableTiming);
    for (int x = 0; x < kXSlots && e == hipSuccess; ++x) {
      e = hipEventCreateWithFlags(&s.ev_keys[x], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev_xdone[x], hipEventDisableTiming);
    }
    for (hipEvent_t* ev : {&s.ev_cdone, &s.ev_rcopy, &s.ev_fork, &s.ev_join, &s.ev_tail[0], &s.ev_tail[1], &s.ev_tail[2],
                           &s.ev_tail[3], &s.ev_tail[4]})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    for (int t = 0; t < kQBufs; ++t)
      for (hipEvent_t* ev : {&s.ev_stage[t], &s.ev_q[t][0], &s.ev_q[t][1]})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      rr_destroy(h);
      return fail(RR_E_HIP, "event setup failed: %s", hipGetErrorString(e));
    }
  }
  // Environment read by the product library: the deadline (RR_TIMEOUT_MS, or its round-3 name RR_DIST_TIMEOUT_MS), the
  // int8 copy's switch and row minimum (RR_SCREEN_I8, RR_SCREEN_I8_MIN_ROWS; include/rag_retrieval.h rr_screen_int8)
  // and RR_HOST_PROF (host-side call timings printed at rr_destroy). Every path setting is an rr_set_option (results
  // unchanged by any of them); the A/B environment (RR_AB_ENV builds only) is below.
  if (const char* e = getenv("RR_DIST_TIMEOUT_MS")) h->timeout_ms = std::max(0, atoi(e));   // (the round-3 name)
  if (const char* e = getenv("RR_TIMEOUT_MS")) h->timeout_ms = std::max(0, atoi(e));
  if (const char* e = getenv("RR_HOST_PROF")) h->host_prof = atoi(e) != 0;
  if (const char* e = getenv("RR_SCREEN_I8")) h->screen_i8 = atoi(e) != 0;
  if (const char* e = getenv("RR_SCREEN_I8_MIN_ROWS")) h->i8_min_rows = std::max<int64_t>(0, atoll(e));
#ifdef RR_AB_ENV
  // A/B builds (tools/ab/build_rev.sh ... "-DRR_AB_ENV=1"; never the product Makefile): every option from RR_<NAME>,
  // and RR_AB_NO_VERIFY, which skips the screened search's verify — INVALID results, for pricing the verify's launch
  for (const OptionDesc& o : kOptions) {
    std::string env = "RR_";
    for (const char* c = o.name; *c; ++c) env += (char)toupper(*c);
    if (const char* e = getenv(env.c_str())) set_option(h, o, atoll(e));
  }
  if (const char* e = getenv("RR_STATIC_SCHEDULE")) h->dyn_sched = atoi(e) == 0;
  if (const char* e = getenv("RR_AB_NO_VERIFY")) h->ab_no_verify = atoi(e) != 0;
#endif
  *out = h;
  return RR_OK;
}

void rr_destroy(rr_handle* h) {
  if (!h) return;
  xw_stop(h);
  if (h->host_prof) {
    static const char* what[10] = {"rr_search_staged", "exchange enqueue", "ncclAllGather call", "screen+verify launches",
                                   "x: ev_keys record", "x: lane waits", "x: merge launch", "x: ev_xdone record",
                                   "c: prep launch", "c: screen launch"};
    for (int i = 0; i < 10; ++i)
      if (h->hp.n[i])
        fprintf(stderr, "[rr host prof] %s: %.2f us x %lld\n", what[i], h->hp.ns[i] / 1e3 / h->hp.n[i],
                (long long)h->hp.n[i]);
  }
  if (h->failed) {
    // device work missed its deadline: an all-gather may still be waiting for a peer. Abort the communicators
    // (their kernels observe the abort and exit) and release nothing else — freeing buffers or destroying streams
    // that queued work may still reference would wait for it, or fault. The process is expected to exit.
    for (Shard& s : h->shards) {
      hipSetDevice(s.dev);
      if (s.comm2) ncclCommAbort(s.comm2);
      if (s.comm) ncclCommAbort(s.comm);
    }
    delete h;
    return;
  }
  for (Shard& s : h->shards) free_shard(s);
  if (h->pin_out) hipHostFree(h->pin_out);
  if (h->pin_q) hipHostFree(h->pin_q);
  for (AsyncSlot& a : h->aslots) {
    if (a.pin) hipHostFree(a.pin);
    if (a.done) hipEventDestroy(a.done);
  }

  delete h;
}

int rr_get_unique_id(char* out) {
  if (!out) return fail(RR_E_INVALID, "out is null");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out, id.internal, RR_UNIQUE_ID_BYTES);
  return RR_OK;
}

int rr_init_dist(rr_handle* h, int world, int rank, const char* unique_id) {
  if (!h || !unique_id) return fail(RR_E_INVALID, "null argument");
  if (h->shards.size() != 1) return fail(RR_E_UNSUPPORTED, "multi-process mode needs exactly one local device");
  if (h->loaded) return fail(RR_E_STATE, "rr_init_dist must precede loading the corpus");
  if (world < 1 || rank < 0 || rank >= world) return fail(RR_E_INVALID, "bad world/rank %d/%d", world, rank);
  if (h->shards[0].comm) return fail(RR_E_STATE, "rr_init_dist already called on this handle");
  // A communicator is created for every world size, 1 included: the search then always takes the RCCL
  // all-gather exchange (with one rank RCCL copies the rank's own candidates), so a 1-GPU box runs the
  // same data path as a node.
  Shard& s = h->shards[0];
  HIP_TRY(hipSetDevice(s.dev));
  ncclUniqueId id;
  memcpy(id.internal, unique_id, RR_UNIQUE_ID_BYTES);
  NCCL_TRY(ncclCommInitRank(&s.comm, world, id, rank));
  NCCL_TRY(ncclCommSplit(s.comm, 0, rank, &s.comm2, nullptr));   // the second exchange lane's communicator
  h->world = world;
  h->shard_base = rank;
  h->dist = true;
  xw_start(h);
  return RR_OK;
}

int rr_dist_info(const rr_handle* h, int* rccl_ranks, int* rccl_rank) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  int n = 0, r = -1;
  if (h->dist && h->shards[0].comm) {
    NCCL_TRY(ncclCommCount(h->shards[0].comm, &n));
    NCCL_TRY(ncclCommUserRank(h->shards[0].comm, &r));
  }
  if (rccl_ranks) *rccl_ranks = n;
  if (rccl_rank) *rccl_rank = r;
  return RR_OK;
}

int rr_load(rr_handle* h, const float* host_corpus, int64_t n, int32_t d) {
  if (!h || !host_corpus) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (int rc = prepare_ranges(h, n, d)) return rc;
  for (Shard& s : h->shards)
    if (s.rows() > 0)
      if (int rc = upload_rows(h, s, host_corpus + s.row_begin * (int64_t)d, 0, s.rows())) return rc;
  if (int rc = finish_all(h)) return rc;
  h->loaded = true;
  return RR_OK;
}

int rr_load_rows(rr_handle* h, const float* host_rows, int64_t row_begin, int64_t n_rows, int64_t n_total,
                 int32_t d) {
  if (!h || !host_rows) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (int rc = prepare_ranges(h, n_total, d)) return rc;
  for (Shard& s : h->shards) {
    if (s.row_begin < row_begin || s.row_end > row_begin + n_rows)
      return fail(RR_E_INVALID, "rows [%lld,%lld) do not cover shard [%lld,%lld)", (long long)row_begin,
                  (long long)(row_begin + n_rows), (long long)s.row_begin, (long long)s.row_end);
    if (s.rows() > 0)
      if (int rc = upload_rows(h, s, host_rows + (s.row_begin - row_begin) * (int64_t)d, 0, s.rows())) return rc;
  }
  if (int rc = finish_all(h)) return rc;
  h->loaded = true;
  return RR_OK;
}

int rr_fill_synthetic(rr_handle* h, int kind, uint64_t seed, int64_t n_total, int32_t d) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (kind != RR_SYNTH_EXACT_INT && kind != RR_SYNTH_UNIT_NORM) return fail(RR_E_INVALID, "bad kind %d", kind);
  if (int rc = prepare_ranges(h, n_total, d)) return rc;
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    const int64_t rows = s.rows();
    if (rows > 0) {
      // generate fp32 rows in chunks, then convert into the storage layout like uploaded rows
      const int64_t chunk_rows = std::max<int64_t>(1, (256ll << 20) / (d * 4));
      float* tmp = nullptr;
      HIP_TRY(hipMalloc((void**)&tmp, (size_t)std::min(chunk_rows, rows) * d * 4));
      for (int64_t r0 = 0; r0 < rows; r0 += chunk_rows) {
        const int64_t nr = std::min(chunk_rows, rows - r0);
        hipError_t e = rr::launch_synth(kind, seed, s.row_begin + r0, nr, d, tmp, s.stream);
        if (e == hipSuccess) e = store_rows(h, s, tmp, r0, nr);
        if (e != hipSuccess) {
          hipFree(tmp);
          return fail(RR_E_HIP, "synthetic fill failed: %s", hipGetErrorString(e));
        }
        if (int rc = wait_stream(h, s, s.stream, "the synthetic fill")) return rc;   // (a timeout fails the handle)
      }
      hipFree(tmp);
    }
  }
  if (int rc = finish_all(h)) return rc;
  h->loaded = true;
  return RR_OK;
}

int rr_info(const rr_handle* h, int64_t* n_total, int32_t* d, int32_t* n_local_shards, int32_t* world_shards) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (n_total) *n_total = h->n_total;
  if (d) *d = h->d;
  if (n_local_shards) *n_local_shards = (int32_t)h->shards.size();
  if (world_shards) *world_shards = h->world;
  return RR_OK;
}

int rr_shard_range(const rr_handle* h, int i, int64_t* begin, int64_t* end) {
  if (!h || i < 0 || i >= (int)h->shards.size()) return fail(RR_E_INVALID, "bad shard %d", i);
  if (begin) *begin = h->shards[i].row_begin;
  if (end) *end = h->shards[i].row_end;
  return RR_OK;
}

int rr_update_rows(rr_handle* h, const float* host_rows, const int64_t* row_idx, int64_t n_rows, int32_t d) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  // Under rr_init_dist this call is a collective (the range agreement below): every rank reaches it, with its own
  // argument checks folded into the agreed value, so a rank that rejects its arguments fails together with its peers
  // instead of leaving them in the allreduce until the deadline.
  int ok = 1;
  if ((!host_rows || !row_idx) && n_rows > 0) ok = fail(RR_E_INVALID, "null argument");
  else if (!h->loaded) ok = fail(RR_E_STATE, "no corpus loaded");
  else if (d != h->d) ok = fail(RR_E_INVALID, "row dim %d != corpus dim %d", d, h->d);
  else if (n_rows < 0) ok = fail(RR_E_INVALID, "n_rows=%lld", (long long)n_rows);
  for (int64_t i = 0; ok == 1 && i < n_rows; ++i)
    if (row_idx[i] < 0 || row_idx[i] >= h->n_total)
      ok = fail(RR_E_INVALID, "row index %lld outside [0, %lld)", (long long)row_idx[i], (long long)h->n_total);
  const int local_rc = ok == 1 ? RR_OK : ok;
  // Whether the rows keep the screen's bound valid (finish_corpus), decided over every given row on the host:
  // fp32 storage, every |x| < 2^15 (the f16 screens' reading); bf16 storage, finite rows of norm < 2^59 (its int8
  // screen's kBf16ScreenNorm, with a margin for the bf16 rounding and the fp32 norm the device computes).
  bool in_range = local_rc == RR_OK;
  if (in_range && h->dtype == RR_DTYPE_BF16) {
    for (int64_t r = 0; r < n_rows && in_range; ++r) {
      double ss = 0.0;
      for (int j = 0; j < d; ++j) ss += (double)host_rows[r * d + j] * host_rows[r * d + j];
      in_range = ss < 0x1p118;   // (NaN: no)
    }
  } else if (in_range) {
    for (int64_t e = 0; e < n_rows * (int64_t)d && in_range; ++e) in_range = fabsf(host_rows[e]) < 32768.0f;   // NaN: no
  }
  // the last search may still be re-run from the rows about to change: settle it, and let every stream drain
  if (local_rc == RR_OK)
    if (int rc = rr_synchronize(h)) return rc;   // (a failed handle: its peers meet the deadline below)
  // agreed across the ranks (an RCCL min): the arguments were valid everywhere, and whether the screen still holds —
  // a rank given other rows than its peers must not keep screening while they stop (the list width sizes the
  // all-gather)
  int agreed[2] = {local_rc == RR_OK ? 1 : 0, in_range ? 1 : 0};
  const std::string why = g_err;
  if (int rc = agree_min(h, agreed, 2, "the ranks' row-update agreement", 10)) return rc;
  if (local_rc != RR_OK) return fail(local_rc, "%s", why.c_str());
  if (!agreed[0]) return fail(RR_E_INVALID, "rank %d of %d: a peer rank rejected its row update arguments",
                              h->shard_base, h->world);
  in_range = agreed[1] != 0;
  const size_t eb = elem_bytes(h->dtype);
  const bool norms = keeps_norms(h) && kdt_of(h->dtype) != rr::KDT_F32_SPLIT;   // (the split computes its own)
  for (Shard& s : h->shards) {
    std::vector<int64_t> mine;
    for (int64_t i = 0; i < n_rows; ++i)
      if (row_idx[i] >= s.row_begin && row_idx[i] < s.row_end) mine.push_back(i);
    if (mine.empty()) continue;
    HIP_TRY(hipSetDevice(s.dev));
    std::vector<float> packed(mine.size() * (size_t)d);
    for (size_t j = 0; j < mine.size(); ++j)
      memcpy(packed.data() + j * d, host_rows + mine[j] * (int64_t)d, (size_t)d * 4);
    float* tmp = nullptr;
    HIP_TRY(hipMalloc((void**)&tmp, packed.size() * 4));
    hipError_t e = hipMemcpyAsync(tmp, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, s.stream);
    // in the given order: a repeated index keeps its last row
    for (size_t j = 0; j < mine.size() && e == hipSuccess; ++j) {
      const int64_t lr = row_idx[mine[j]] - s.row_begin;
      e = store_rows(h, s, tmp + j * d, lr, 1);
      if (e == hipSuccess && norms)
        e = rr::launch_row_norms(h->dtype == RR_DTYPE_BF16 ? 1 : 0, (const char*)s.corpus + lr * d * eb, 1, d,
                                 s.norms + lr, s.stream);
    }
    if (e != hipSuccess) {
      hipFree(tmp);
      return fail(RR_E_HIP, "row update failed: %s", hipGetErrorString(e));
    }
    if (int rc = wait_stream(h, s, s.stream, "the row update")) return rc;
    hipFree(tmp);
  }
  if (!in_range) h->screen_ok = false;
  return RR_OK;
}

int rr_read_rows(const rr_handle* h, int64_t row_begin, int64_t n_rows, float* host_out) {
  if (!h || !host_out) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (!h->loaded) return fail(RR_E_STATE, "no corpus loaded");
  const int d = h->d;
  int64_t done = 0;
  while (done < n_rows) {
    const int64_t row = row_begin + done;
    const Shard* sp = nullptr;
    for (const Shard& s : h->shards)
      if (row >= s.row_begin && row < s.row_end) sp = &s;
    if (!sp) return fail(RR_E_INVALID, "row %lld is not held locally", (long long)row);
    const int64_t nr = std::min(n_rows - done, sp->row_end - row);
    const int64_t lr = row - sp->row_begin;
    HIP_TRY(hipSetDevice(sp->dev));
    {
      float* tmp = nullptr;
      HIP_TRY(hipMalloc((void**)&tmp, (size_t)nr * d * 4));
      const int kdt = kdt_of(h->dtype);
      hipError_t e =
          kdt == rr::KDT_BF16
              ? rr::launch_bf16_to_f32((const uint16_t*)sp->corpus + lr * d, tmp, nr, d, sp->stream)
          : kdt == rr::KDT_F32_SPLIT
              ? rr::launch_unsplit_f32((const float*)sp->corpus + lr * d, sp->rscale + lr, nr, d, tmp, sp->stream)
              : rr::launch_permute_f32((const float*)sp->corpus + lr * d, tmp, nr, d, 1, sp->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(sp->stream);
      if (e == hipSuccess) e = hipMemcpy(host_out + done * d, tmp, (size_t)nr * d * 4, hipMemcpyDeviceToHost);
      hipFree(tmp);
      if (e != hipSuccess) return fail(RR_E_HIP, "read_rows failed: %s", hipGetErrorString(e));
    }
    done += nr;
  }
  return RR_OK;
}

int rr_screen_factors(rr_handle* h, int64_t row_begin, int64_t n_rows, float* norms, float* scales,
                      float* err_norms) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (!h->loaded) return fail(RR_E_STATE, "no corpus loaded");
  if (n_rows < 0) return fail(RR_E_INVALID, "n_rows=%lld", (long long)n_rows);
  if (int rc = rr_synchronize(h)) return rc;   // (a row update or a load may still be writing them)
  int64_t done = 0;
  while (done < n_rows) {
    const int64_t row = row_begin + done;
    Shard* sp = nullptr;
    for (Shard& s : h->shards)
      if (row >= s.row_begin && row < s.row_end) sp = &s;
    if (!sp) return fail(RR_E_INVALID, "row %lld is not held locally", (long long)row);
    if ((scales || err_norms) && !sp->scr8)
      return fail(RR_E_STATE, "the shard holding row %lld has no int8 copy", (long long)row);
    const int64_t nr = std::min(n_rows - done, sp->row_end - row);
    const int64_t lr = row - sp->row_begin;
    HIP_TRY(hipSetDevice(sp->dev));
    if (norms) HIP_TRY(hipMemcpy(norms + done, sp->norms + lr, (size_t)nr * 4, hipMemcpyDeviceToHost));
    if (scales) HIP_TRY(hipMemcpy(scales + done, sp->sx8 + lr, (size_t)nr * 4, hipMemcpyDeviceToHost));
    if (err_norms) HIP_TRY(hipMemcpy(err_norms + done, sp->e8 + lr, (size_t)nr * 4, hipMemcpyDeviceToHost));
    done += nr;
  }
  return RR_OK;
}

int rr_set_queries(rr_handle* h, const float* host_q, int32_t b, int32_t d) {
  if (!h || (!host_q && b > 0)) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (!h->loaded) return fail(RR_E_STATE, "no corpus loaded");
  if (d != h->d) return fail(RR_E_INVALID, "query dim %d != corpus dim %d", d, h->d);
  if (b < 1) return fail(RR_E_INVALID, "b=%d", b);
  if (int rc = ensure_buffers(h, b, 1)) return rc;
  // stage through a pinned buffer per shard (the copy is then a plain async DMA); a buffer is rewritten
  // only after the previous batch's copy out of it has completed
  const size_t qbytes = (size_t)b * d * 4;
  for (Shard& s : h->shards) {   // every shard's copy out of pin_q has landed before it is rewritten
    HIP_TRY(hipSetDevice(s.dev));
    if (s.pin_q_free) {
      if (int rc = wait_event(h, s, s.pin_q_free, "the previous batch's query copy")) return rc;
    } else {
      HIP_TRY(hipEventCreateWithFlags(&s.pin_q_free, hipEventDisableTiming));
    }
  }
  if (qbytes > h->pin_q_cap) {
    if (h->pin_q) HIP_TRY(hipHostFree(h->pin_q));
    h->pin_q = nullptr;
    h->pin_q_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&h->pin_q, qbytes, hipHostMallocDefault));
    h->pin_q_cap = qbytes;
  }
  memcpy(h->pin_q, host_q, qbytes);
  int nq = 0;
  if (int rc = begin_stage(h, &nq)) return rc;
  if (int rc = stage_queries(h, nq, h->pin_q, b, -1, true)) return rc;
  h->qpar = nq;
  h->cur_b = b;
  return RR_OK;
}

int rr_set_queries_device(rr_handle* h, const float* dev_q, int32_t b, int32_t d) {
  if (!h || !dev_q) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (!h->loaded) return fail(RR_E_STATE, "no corpus loaded");
  if (d != h->d) return fail(RR_E_INVALID, "query dim %d != corpus dim %d", d, h->d);
  if (b < 1) return fail(RR_E_INVALID, "b=%d", b);
  if (int rc = ensure_buffers(h, b, 1)) return rc;
  const int src_dev = h->shards[0].dev;
  int nq = 0;
  if (int rc = begin_stage(h, &nq)) return rc;
  if (int rc = stage_queries(h, nq, dev_q, b, src_dev, false)) return rc;
  h->qpar = nq;
  h->cur_b = b;
  return RR_OK;
}

static int search_staged_body(rr_handle* h, int32_t k);
int rr_search_staged(rr_handle* h, int32_t k) {
  if (!h || !h->host_prof) return search_staged_body(h, k);
  const int64_t t0 = now_ns();
  const int rc = search_staged_body(h, k);
  h->hp.ns[0] += now_ns() - t0;
  ++h->hp.n[0];
  return rc;
}
static int search_staged_body(rr_handle* h, int32_t k) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (!h->loaded || h->cur_b < 1) return fail(RR_E_STATE, "no queries staged");
  if (k < 1) return fail(RR_E_INVALID, "k=%d must be >= 1", k);
  const int b = h->cur_b;
  if (int rc = ensure_buffers(h, b, k)) return rc;
  const int slots = block_slots(h, b, k);
  h->last_screened = checked(h, k, slots);
  h->last_narrow = screened(h, k, slots) && narrow_lists(h, k);
  h->last_full = h->full_lists;
  h->last_wide = h->screen_wide;
  // judged by the int8 rule only when every shard (of every rank) screened the int8 copy: rank-consistent
  h->last_i8 = i8_active(h) && h->i8_all;
  h->last_blocks = screened(h, k, slots) ? (b + slots - 1) / slots : 0;
  h->last_seq0 = h->screen_seq + 1;
  h->last_settled = !h->last_screened;
  h->last_qpar = h->qpar;
  const bool paused = h->screen_pause > 0 && h->kernel == RR_KERNEL_AUTO;
  for (int q0 = 0; q0 < b; q0 += slots) {
    const int bb = std::min(slots, b - q0);
    if (int rc = enqueue_block(h, q0, bb, k, slots)) return rc;
  }
  if (paused) pause_tick(h, (b + slots - 1) / slots);
  h->last_k = k;
  h->last_b = b;
  return RR_OK;
}

int rr_screen_state(rr_handle* h, int32_t* full_lists, int64_t* pause_left, int64_t* pauses) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (full_lists) *full_lists = h->full_lists ? 1 : 0;
  if (pause_left) *pause_left = h->screen_pause;
  if (pauses) *pauses = h->pauses;
  return RR_OK;
}

int rr_last_shape(const rr_handle* h, int32_t* b, int32_t* k) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (b) *b = h->last_b;
  if (k) *k = h->last_k;
  return RR_OK;
}

namespace {

int sync_streams(rr_handle* h) {
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    for (hipStream_t st : {s.stream, s.xstream, s.xstream2, s.cstream2, s.sstream})
      if (st)
        if (int rc = wait_stream(h, s, st)) return rc;
    s.c2_busy = false;
    s.rcopy_pending = false;
  }
  return collect_timing(h);
}

// rr_screen_counts' D2H copies on shard s's `stream`: its counters, and for shard 0 the flag word (`flag`: the last
// search is unsettled), into its pinned staging
hipError_t queue_count_copies(const rr_handle* h, Shard& s, bool flag) {
  if (!s.pin_scount) return hipSuccess;
  hipError_t e = hipSuccess;
  if (s.scount) e = hipMemcpyAsync(s.pin_scount, s.scount, 4 * sizeof(int), hipMemcpyDeviceToHost, s.stream);
  if (e == hipSuccess && flag && &s == &h->shards[0] && s.out_base)
    e = hipMemcpyAsync(s.pin_scount + 4, s.out_base, sizeof(uint64_t), hipMemcpyDeviceToHost, s.stream);
  return e;
}
// sync_streams ending on records at every stream's tail (Shard::ev_tail): the other streams' records are queued
// together and waited on together with `stream`'s work; then, every stream idle (the flag word and the counters may
// be written on any of them), the count copies on `stream` (queue_count_copies) and its own tail record.
int sync_streams_tail(rr_handle* h, bool flag) {
  if (h->xw)   // every posted exchange issued: its launches precede the records
    if (int rc = xw_drain(h)) return rc;
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    const hipStream_t others[4] = {s.xstream, s.xstream2, s.cstream2, s.sstream};
    for (int i = 1; i < 5; ++i)
      if (others[i - 1]) HIP_TRY(hipEventRecord(s.ev_tail[i], others[i - 1]));
  }
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    for (int i = 1; i < (s.sstream ? 5 : 4); ++i)
      if (int rc = wait_event(h, s, s.ev_tail[i], "device work (stream tails)")) return rc;
    HIP_TRY(queue_count_copies(h, s, flag));
    HIP_TRY(hipEventRecord(s.ev_tail[0], s.stream));
  }
  for (Shard& s : h->shards) {
    HIP_TRY(hipSetDevice(s.dev));
    if (int rc = wait_event(h, s, s.ev_tail[0], "device work and the screened-search counts")) return rc;
    s.c2_busy = false;
    s.rcopy_pending = false;
  }
  return collect_timing(h);
}

// D2H of device bytes on local shard 0's `stream` (never the null stream: it sits in the normal-priority queue pool
// with RCCL's internal streams, whose barrier packets may wait for an all-gather). The streams are idle.
int copy_out(rr_handle* h, void* dst, const void* src, size_t bytes) {
  Shard& s = h->shards[0];
  HIP_TRY(hipSetDevice(s.dev));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s.stream));
  return wait_stream(h, s, s.stream, "result copy");
}

// Screened search, last step: `flag` is the last search's flag word (shard 0's result head, which after an
// exchange holds the largest flag of every shard, so every rank sees the same value). When a block of that
// search was flagged, re-run the search — its queries are still staged — with the one-pass exact kernel.
int settle_screen(rr_handle* h, uint64_t flag, bool* rerun) {
  *rerun = false;
  if (!h->last_screened || h->last_settled) return RR_OK;
  h->last_settled = true;
  const bool flagged = flag >= (uint64_t)h->last_seq0;
  observe_settled(h, h->last_blocks, h->last_narrow, h->last_full, h->last_wide, h->last_i8, flagged);
  if (!flagged) return RR_OK;
  // the search's own queries (begin_stage keeps its buffer intact until it is settled); a batch staged
  // since stays staged
  const int saved_kernel = h->kernel, saved_qpar = h->qpar, saved_b = h->cur_b;
  h->kernel = RR_KERNEL_EXACT;
  h->qpar = h->last_qpar;
  h->cur_b = h->last_b;
  const int rc = rr_search_staged(h, h->last_k);
  h->kernel = saved_kernel;
  h->qpar = saved_qpar;
  h->cur_b = saved_b;
  if (rc) return rc;
  ++h->screen_reruns;
  *rerun = true;
  return sync_streams(h);
}

// (through pinned staging when there is one: a D2H copy into pageable memory costs the runtime a staged copy)
int read_flag(rr_handle* h, uint64_t* flag) {
  Shard& s = h->shards[0];
  *flag = 0;
  if (!s.out_base) return RR_OK;
  if (!s.pin_scount) return copy_out(h, flag, s.out_base, sizeof(uint64_t));
  if (int rc = copy_out(h, s.pin_scount + 4, s.out_base, sizeof(uint64_t))) return rc;
  memcpy(flag, (const void*)(s.pin_scount + 4), sizeof(uint64_t));
  return RR_OK;
}

}  // namespace

int rr_synchronize(rr_handle* h) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (int rc = sync_streams(h)) return rc;
  if (!h->last_screened || h->last_settled) return RR_OK;   // (settled: nothing to read)
  uint64_t flag = 0;
  if (int rc = read_flag(h, &flag)) return rc;
  bool rerun = false;
  return settle_screen(h, flag, &rerun);
}

int rr_fetch_results(rr_handle* h, float* out_scores, int64_t* out_idx) {
  if (!h || !out_scores || !out_idx) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (h->last_k < 1) return fail(RR_E_STATE, "no search has run");
  if (int rc = sync_streams(h)) return rc;
  Shard& s = h->shards[0];
  const size_t cnt = (size_t)h->last_b * h->last_k;
  const size_t span = s.out_off + cnt * 8;
  for (int attempt = 0; attempt < 2; ++attempt) {
    HIP_TRY(hipSetDevice(s.dev));
    uint64_t flag = 0;
    if (s.out_off > (1u << 20)) {   // capacity grown far beyond this search: plain copies
      if (int rc = copy_out(h, out_scores, s.out_scores, cnt * 4)) return rc;
      if (int rc = copy_out(h, out_idx, s.out_idx, cnt * 8)) return rc;
      if (int rc = read_flag(h, &flag)) return rc;
    } else {
      if (span > h->pin_out_cap) {
        if (h->pin_out) HIP_TRY(hipHostFree(h->pin_out));
        h->pin_out = nullptr;
        h->pin_out_cap = 0;
        HIP_TRY(hipHostMalloc((void**)&h->pin_out, span, hipHostMallocDefault));
        h->pin_out_cap = span;
      }
      // one pinned D2H of [flag word | scores | pad | indices] (the streams are idle)
      if (int rc = copy_out(h, h->pin_out, s.out_base, span)) return rc;
      memcpy(&flag, h->pin_out, sizeof flag);
      memcpy(out_scores, h->pin_out + kOutHead, cnt * 4);
      memcpy(out_idx, h->pin_out + s.out_off, cnt * 8);
    }
    bool rerun = false;
    if (int rc = settle_screen(h, flag, &rerun)) return rc;
    if (!rerun) return RR_OK;
  }
  return RR_OK;
}

int rr_search(rr_handle* h, const float* host_q, int32_t b, int32_t d, int32_t k, float* out_scores,
              int64_t* out_idx) {
  if (int rc = rr_set_queries(h, host_q, b, d)) return rc;
  if (int rc = rr_search_staged(h, k)) return rc;
  return rr_fetch_results(h, out_scores, out_idx);
}

int rr_search_async(rr_handle* h, const float* host_q, int32_t b, int32_t d, int32_t k, int32_t* ticket) {
  if (!h || !host_q || !ticket) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (!h->loaded) return fail(RR_E_STATE, "no corpus loaded");
  if (d != h->d) return fail(RR_E_INVALID, "query dim %d != corpus dim %d", d, h->d);
  if (b < 1 || k < 1) return fail(RR_E_INVALID, "b=%d k=%d", b, k);
  const int32_t t = h->next_ticket;
  AsyncSlot& a = h->aslots[t % kAsyncSlots];
  if (a.pending) return fail(RR_E_STATE, "%d searches in flight: rr_wait(%d) first", kAsyncSlots, a.ticket);
  if (int rc = ensure_buffers(h, b, k)) return rc;
  // pinned slot: [queries | flag word | scores | pad | indices]; the queries stay for a possible re-run
  const size_t qbytes = (size_t)b * d * 4, cnt = (size_t)b * k;
  const size_t res_off = (qbytes + 255) & ~(size_t)255;
  const size_t idx_off = res_off + ((kOutHead + cnt * 4 + 255) & ~(size_t)255);
  const size_t need = idx_off + cnt * 8;
  if (need > a.cap) {
    if (a.pin) HIP_TRY(hipHostFree(a.pin));
    a.pin = nullptr;
    a.cap = 0;
    HIP_TRY(hipHostMalloc((void**)&a.pin, need, hipHostMallocDefault));
    a.cap = need;
  }
  if (!a.done) HIP_TRY(hipEventCreateWithFlags(&a.done, hipEventDisableTiming));
  memcpy(a.pin, host_q, qbytes);
  int nq = 0;
  if (int rc = begin_stage(h, &nq)) return rc;
  if (int rc = stage_queries(h, nq, a.pin, b, -1, false)) return rc;
  h->qpar = nq;
  h->cur_b = b;
  if (int rc = rr_search_staged(h, k)) return rc;
  // results come back on the stream that wrote them last: the exchange stream when there is an exchange
  // (the serial k > 32 exchange also orders it after itself), else the compute stream
  Shard& s0 = h->shards[0];
  HIP_TRY(hipSetDevice(s0.dev));
  const bool xchg = h->world > 1 || h->dist;
  if (int rc = xw_drain(h)) return rc;   // (last_x, rcopy: the exchange state is the caller's once drained)
  // without an exchange: after a screened search, on the stream of its last verify (the copy then holds back the
  // next verify on the other stream, which rewrites the rows: ev_q re-recorded below); else on `stream`
  const bool on_v = !xchg && h->last_scr_block && s0.last_vsi >= 0;
  hipStream_t rs = xchg ? (s0.last_x > 0 && (s0.last_x & 1) ? s0.xstream2 : s0.xstream)   // the last merge's lane
                        : on_v ? stream_of(s0, s0.last_vsi) : s0.stream;
  if (!xchg && !on_v)
    if (int rc = join_main(s0)) return rc;
  HIP_TRY(hipMemcpyAsync(a.pin + res_off, s0.out_base, kOutHead, hipMemcpyDeviceToHost, rs));
  HIP_TRY(hipMemcpyAsync(a.pin + res_off + kOutHead, s0.out_scores, cnt * 4, hipMemcpyDeviceToHost, rs));
  HIP_TRY(hipMemcpyAsync(a.pin + idx_off, s0.out_idx, cnt * 8, hipMemcpyDeviceToHost, rs));
  HIP_TRY(hipEventRecord(a.done, rs));
  // the next writer of these result rows on another stream must wait for the copy: the next screened verify on the
  // other compute stream (ev_q), a cstream2 block after a search on `stream` (ev_fork), an exchange merge on the other
  // lane or a serial exchange on `stream` (ev_rcopy)
  if (on_v) {
    HIP_TRY(hipEventRecord(s0.ev_q[s0.last_vq][s0.last_vsi], rs));
    s0.evq_alias[s0.last_vq][s0.last_vsi] = nullptr;
  }
  if (!xchg && !on_v) {
    if (int rc = fork_point(s0)) return rc;
  }
  if (xchg) {
    HIP_TRY(hipEventRecord(s0.ev_rcopy, rs));
    s0.rcopy_pending = true;
  }
  a.b = b;
  a.k = k;
  a.ticket = t;
  a.screened = h->last_screened;
  a.narrow = h->last_narrow;
  a.i8 = h->last_i8;
  a.full = h->last_full;
  a.wide = h->last_wide;
  a.blocks = h->last_blocks;
  a.seq0 = h->last_seq0;
  a.pending = true;
  h->next_ticket = t + 1 < 0x40000000 ? t + 1 : 0;
  *ticket = t;
  return RR_OK;
}

int rr_wait(rr_handle* h, int32_t ticket, float* out_scores, int64_t* out_idx) {
  if (!h || !out_scores || !out_idx) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (ticket < 0) return fail(RR_E_INVALID, "bad ticket %d", ticket);
  AsyncSlot& a = h->aslots[ticket % kAsyncSlots];
  if (!a.pending || a.ticket != ticket) return fail(RR_E_STATE, "ticket %d is not in flight", ticket);
  if (int rc = wait_event(h, h->shards[0], a.done, "an asynchronous search")) return rc;
  a.pending = false;
  const size_t qbytes = (size_t)a.b * h->d * 4, cnt = (size_t)a.b * a.k;
  const size_t res_off = (qbytes + 255) & ~(size_t)255;
  const size_t idx_off = res_off + ((kOutHead + cnt * 4 + 255) & ~(size_t)255);
  uint64_t flag = 0;
  memcpy(&flag, a.pin + res_off, sizeof flag);
  if (a.screened) observe_settled(h, a.blocks, a.narrow, a.full, a.wide, a.i8, flag >= (uint64_t)a.seq0);
  // this ticket's search, if it is still the handle's last one, is settled here: a later rr_synchronize /
  // rr_fetch_results must neither observe it again nor re-run it a second time
  if (a.screened && h->last_screened && !h->last_settled && h->last_seq0 == a.seq0) h->last_settled = true;
  if (a.screened && flag >= (uint64_t)a.seq0) {
    // a block needed the exact pass: this batch again, exactly (every rank of an exchange sees the same
    // flag here, so all re-run it together). A batch staged with rr_set_queries before this wait stays the
    // staged batch (the re-run goes through the other query buffer).
    if (int rc = sync_streams(h)) return rc;
    const int saved_qpar = h->qpar, saved_b = h->cur_b;
    int nq = 0;
    if (int rc = begin_stage(h, &nq)) return rc;
    if (int rc = stage_queries(h, nq, a.pin, a.b, -1, false)) return rc;
    h->qpar = nq;
    h->cur_b = a.b;
    const int saved = h->kernel;
    h->kernel = RR_KERNEL_EXACT;
    int rc = rr_search_staged(h, a.k);
    h->kernel = saved;
    if (rc == RR_OK) {
      ++h->screen_reruns;
      rc = rr_fetch_results(h, out_scores, out_idx);
    }
    h->qpar = saved_qpar;
    h->cur_b = saved_b;
    return rc;
  }
  memcpy(out_scores, a.pin + res_off + kOutHead, cnt * 4);
  memcpy(out_idx, a.pin + idx_off, cnt * 8);
  return collect_timing(h);
}

// As rr_synchronize, then the counters: the last search's flag word and every shard's counters come back in the same
// wait as the streams' work (sync_streams_tail; the end of a timed window pays this call, bench.py timed_steps). A
// re-run the flag asks for counts nothing (the exact kernel does not screen); settle_screen waits for it.
int rr_screen_counts(rr_handle* h, int64_t* blocks, int64_t* flagged, int64_t* reruns, int64_t* wide_slots) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  const bool unsettled = h->last_screened && !h->last_settled;
  // every stream idle, with shard 0's flag word (pinned) and each shard's counters copied behind its work
  if (int rc = sync_streams_tail(h, unsettled)) return rc;
  int64_t fb = 0, ws = 0;
  uint64_t flag = 0;
  for (Shard& s : h->shards) {
    if (!s.scount || !s.pin_scount) continue;
    fb += ((volatile int*)s.pin_scount)[0];
    ws += ((volatile int*)s.pin_scount)[2];   // (wcount = scount + 2)
  }
  if (unsettled) {
    Shard& s0 = h->shards[0];
    if (s0.out_base && s0.pin_scount) memcpy(&flag, (const void*)(s0.pin_scount + 4), sizeof flag);
    else if (int rc = read_flag(h, &flag)) return rc;
    bool rerun = false;
    if (int rc = settle_screen(h, flag, &rerun)) return rc;
  }
  if (blocks) *blocks = h->screen_blocks * (int64_t)h->shards.size();
  if (flagged) *flagged = fb;
  if (reruns) *reruns = h->screen_reruns;
  if (wide_slots) *wide_slots = ws;
  return RR_OK;
}

int rr_screen_repairs(rr_handle* h, int64_t* repaired_slots) {
  if (!h || !repaired_slots) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  if (int rc = rr_synchronize(h)) return rc;
  int64_t n = 0;
  for (Shard& s : h->shards) {
    if (!s.wcount) continue;
    HIP_TRY(hipSetDevice(s.dev));
    HIP_TRY(hipMemcpyAsync(s.pin_scount, s.wcount + 1, sizeof(int), hipMemcpyDeviceToHost, s.stream));
    if (int rc = wait_stream(h, s, s.stream, "the repaired-slot count")) return rc;
    n += *(volatile int*)s.pin_scount;
  }
  *repaired_slots = n;
  return RR_OK;
}

int rr_screen_stats(rr_handle* h, int64_t* blocks, int64_t* fallbacks) {
  return rr_screen_counts(h, blocks, fallbacks, nullptr, nullptr);
}

int rr_set_timeout(rr_handle* h, int32_t ms) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (ms < 0) return fail(RR_E_INVALID, "timeout %d ms", ms);
  h->timeout_ms = ms;
  return RR_OK;
}

int rr_stream_queues(rr_handle* h, int i, uint64_t* out) {
  if (!h || !out) return fail(RR_E_INVALID, "null argument");
  if (i < 0 || i >= (int)h->shards.size()) return fail(RR_E_INVALID, "bad shard %d", i);
  if (h->failed) return failed_handle();
  if (int rc = sync_streams(h)) return rc;
  Shard& s = h->shards[i];
  HIP_TRY(hipSetDevice(s.dev));
  uint64_t* dq = nullptr;
  HIP_TRY(hipMalloc((void**)&dq, 5 * sizeof(uint64_t)));
  const hipStream_t st[5] = {s.stream, s.cstream2, s.xstream, s.xstream2, s.sstream};
  hipError_t e = hipSuccess;
  for (int j = 0; j < 5 && e == hipSuccess; ++j)
    if (st[j]) e = rr::launch_queue_probe(dq + j, st[j]);
  int rc = RR_OK;
  if (e == hipSuccess) rc = sync_streams(h);
  if (e == hipSuccess && rc == RR_OK) e = hipMemcpy(out, dq, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  for (int j = 0; j < 5; ++j)
    if (!st[j]) out[j] = 0;   // (no staging stream: stage_stream 0)
  if (!h->failed) hipFree(dq);
  if (rc) return rc;
  if (e != hipSuccess) return fail(RR_E_HIP, "queue probe failed: %s", hipGetErrorString(e));
  return RR_OK;
}

int rr_set_kernel(rr_handle* h, int kernel) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (kernel < RR_KERNEL_AUTO || kernel > RR_KERNEL_SCREEN_FALLBACK) return fail(RR_E_INVALID, "bad kernel %d", kernel);
  h->kernel = kernel;
  return RR_OK;
}

int rr_set_schedule(rr_handle* h, int dynamic) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (int rc = sync_streams(h)) return rc;   // no launch in flight uses the counter
  h->dyn_sched = dynamic ? 1 : 0;
  return RR_OK;
}

int rr_set_compute_streams(rr_handle* h, int32_t n, int32_t* in_use) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (n < -1 || n == 0 || n > 2) return fail(RR_E_INVALID, "compute streams %d (-1 = as is, 1, 2)", n);
  if (n > 0 && n != h->streams) {
    if (int rc = rr_synchronize(h)) return rc;
    for (Shard& s : h->shards) s.last_vsi = -1;
    h->streams = n;
  }
  if (in_use) *in_use = h->shards.empty() ? 1 : (two_streams(h, h->shards[0]) ? 2 : 1);
  return RR_OK;
}

int rr_screen_copy(rr_handle* h, int32_t use, int32_t* present) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (use >= 0) {
    h->screen_copy = use ? 1 : 0;
    if (!use)   // every stream of the handle may still be screening from the copy
      if (int rc = sync_streams(h)) return rc;
    if (!use)
      for (Shard& s : h->shards) {
        HIP_TRY(hipSetDevice(s.dev));
        free_i8(s);
        if (s.scr16) {
          HIP_TRY(hipFree(s.scr16));
          s.scr16 = nullptr;
        }
      }
  }
  if (present) {
    bool all = !h->shards.empty();
    const bool bf = h->dtype == RR_DTYPE_BF16;   // (bf16 storage: its int8 copy)
    for (const Shard& s : h->shards) all = all && ((bf ? s.scr8 != nullptr : s.scr16 != nullptr) || s.rows() == 0);
    *present = all && h->screen_copy && h->loaded ? 1 : 0;
  }
  return RR_OK;
}

int rr_screen_int8(rr_handle* h, int32_t use, int32_t* active) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (use >= 0) {
    h->screen_i8 = use ? 1 : 0;
    // (a copy exists only if the handle loaded with it on)
  }
  if (active) {
    bool all = !h->shards.empty();
    const bool bf = h->dtype == RR_DTYPE_BF16;   // (bf16 storage: no f16 copy)
    for (const Shard& s : h->shards)
      all = all && ((s.scr8 != nullptr && (bf || s.scr16 != nullptr)) || s.rows() == 0);
    *active = all && i8_active(h) && h->loaded ? 1 : 0;
  }
  return RR_OK;
}

int rr_set_option(rr_handle* h, const char* name, int64_t value) {
  if (!h || !name) return fail(RR_E_INVALID, "null argument");
  if (h->failed) return failed_handle();
  const OptionDesc* o = find_option(name);
  if (!o) return fail(RR_E_INVALID, "unknown option '%s'", name);
  if (int rc = rr_synchronize(h)) return rc;   // no search in flight runs under the old setting
  return set_option(h, *o, value);
}

int rr_get_option(const rr_handle* h, const char* name, int64_t* value) {
  if (!h || !name || !value) return fail(RR_E_INVALID, "null argument");
  const OptionDesc* o = find_option(name);
  if (!o) return fail(RR_E_INVALID, "unknown option '%s'", name);
  rr_handle* m = const_cast<rr_handle*>(h);   // (the accessors are shared with the setter; nothing is written)
  if (strcmp(name, "screen_full_lists") == 0) *value = h->full_lists_env ? 1 : 0;
  else if (int64_t* f = option_field64(m, name)) *value = *f;
  else *value = *option_field(m, name);
  return RR_OK;
}

const char* rr_build_info(void) {
#ifdef RR_AB_ENV
  return "gfx950; A/B build (RR_AB_ENV: options from RR_<NAME>, RR_AB_NO_VERIFY)";
#else
  return "gfx950; product build";
#endif
}

int rr_set_timing(rr_handle* h, int enable) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  h->timing = enable != 0;
  return RR_OK;
}

int rr_kernel_time(rr_handle* h, double* total_ms, int64_t* launches, int reset) {
  if (!h) return fail(RR_E_INVALID, "null handle");
  if (h->failed) return failed_handle();
  if (int rc = rr_synchronize(h)) return rc;
  if (total_ms) *total_ms = h->t_ms;
  if (launches) *launches = h->t_count;
  if (reset) {
    h->t_ms = 0.0;
    h->t_count = 0;
  }
  return RR_OK;
}

}  // extern "C"
