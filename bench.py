#!/usr/bin/env python3
"""Benchmark of the MI355X retrieval hot path (BASELINE.json configs[1]: 1M synthetic docs, d=1024,
batch 32, top-k 5, fused similarity + top-k through the C-ABI).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp32|bf16] [--metric cosine|dot]

N > 1 runs one process per GPU. Under torch.distributed.run (RANK/WORLD_SIZE set) this process is one
rank; started plainly (`python bench.py --gpus N`), it launches `python -m torch.distributed.run
--nproc-per-node N --master-addr 127.0.0.1 ... bench.py` as a CHILD before touching any GPU and exits
with its status (no exec).

A step = one batch of B queries through the whole device pipeline (fused MFMA similarity + top-k over
the rank's corpus shard, per-shard merge, RCCL all-gather of candidates over the rank's shard group, final
merge), with the queries already resident in HBM. The corpus (N_DOCS x d) is generated on device. N > 1:
the ranks form R replica groups of S ranks (`--shard-group`, auto: the fewest ranks whose row shards keep
>= 500k rows — 1M docs: S = 2); each group holds the whole corpus as S row shards and searches its own
batches, and `value` counts every group's batches. With R > 1 the same loop over all N ranks as one
row-sharded group is measured too (`row_shard_all`). Rank 0 prints ONE JSON line.

Also reported: host-inclusive latency (H2D of the queries + pipeline + D2H of results) p50/p99 over
synchronous batches, and the CPU baseline = the oracle's restatement of the reference SimpleRetriever
(per-query fp32 matvec + argpartition + argsort) timed on the host cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "retrieval queries/sec + p99 latency, batch=32, 1M docs d=1024, 1/2/4/8 GPU"
SCORE_KERNEL_DOC = ("the corpus-streaming kernel: sk_score_kernel MODE 0 (split-K, LDS-DMA; for fp32 storage the "
                    "screened search's screen — over the int8 screening copy (d a multiple of 512 up to 1024) DT 9 with "
                    "one int8 query piece on 400k-4M-row shards outside repair mode, else DT 8 with two, "
                    "DT 7 over the f16 copy, else DT 6 over the fp32 rows — whose exact fp32 verify of the candidates "
                    "runs on the other compute stream; for bf16 storage DT 9 over the int8 copy of the bf16 rows, verified by "
                    "the bf16 pass's own arithmetic), else fused_score_kernel")


def is_score_kernel(name: str) -> bool:
    """The corpus-streaming launches: sk_score_kernel<DT, NS, KT, COS, RS, QH, MODE, SCHED> with MODE 0 (MODE 1
    is the screened search's 32-workgroup verify), or fused_score_kernel."""
    if "fused_score_kernel" in name:
        return True
    if "sk_score_kernel<" not in name:
        return False
    targs = name.split("sk_score_kernel<", 1)[1].split(">", 1)[0].split(",")
    return len(targs) >= 7 and targs[6].strip() == "0"


def stream_priority_range():
    """(least, greatest) stream priority of the HIP runtime (hipDeviceGetStreamPriorityRange): the library's search
    streams take the greatest, its staging stream the least — separate hardware-queue pools when they differ from the
    normal priority (0) RCCL's and torch's streams use."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        lo, hi = ctypes.c_int(), ctypes.c_int()
        if hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)) != 0:
            return None
        return [lo.value, hi.value]
    except OSError:
        return None


def host_cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n_docs: int, d: int, batch: int, k: int, budget_s: float) -> dict:
    """The reference algorithm on the host: the oracle restatement of
    SimpleRetriever.batch_retrieve (retriever.py:131-166: per-query fp32 sgemv + argpartition + argsort)
    over a bounded sample of batches (as many as fit `budget_s`, at least one), on every core this process
    may run on, plus the stronger batched point (one Q @ A.T sgemm per batch + per-row argpartition)."""
    from threadpoolctl import threadpool_info, threadpool_limits
    from oracle import synth
    from oracle.retriever_oracle import simple_batch_retrieve
    # every core this process may use: its affinity set, capped by the CPU share the host grants it
    # (OMP_NUM_THREADS; 16 per GPU on the MI355X pool, whose os.cpu_count() shows the whole machine)
    cores = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        cores = min(cores, int(os.environ["OMP_NUM_THREADS"]))
    corpus = synth.unit_norm_gaussian(4321, n_docs, d)
    q = synth.unit_norm_gaussian(8765, batch * 64, d)
    with threadpool_limits(limits=cores):
        blas = [{"api": i.get("internal_api"), "version": i.get("version"), "threads": i.get("num_threads")}
                for i in threadpool_info()]
        simple_batch_retrieve(corpus, q[:2], [k, k])            # warm
        t0 = time.perf_counter()
        nb = 0
        while nb < 64 and (nb == 0 or time.perf_counter() - t0 < budget_s):
            simple_batch_retrieve(corpus, q[nb * batch:(nb + 1) * batch], [k] * batch)
            nb += 1
        dt = time.perf_counter() - t0
        # batched variant: one sgemm for the whole batch, then the same per-row top-k selection
        t1 = time.perf_counter()
        nb2 = 0
        while nb2 < 64 and (nb2 == 0 or time.perf_counter() - t1 < budget_s / 3):
            qb = q[nb2 * batch:(nb2 + 1) * batch]
            sims = qb @ corpus.T
            top = np.argpartition(sims, -k, axis=1)[:, -k:]
            np.take_along_axis(top, np.argsort(-np.take_along_axis(sims, top, axis=1), axis=1), axis=1)
            nb2 += 1
        dt2 = time.perf_counter() - t1
    return {"value": round(batch * nb / dt, 3), "unit": "queries/s", "cores": cores, "kind": "port",
            "cpu_model": host_cpu_model(), "os_cpu_count": os.cpu_count(), "blas": blas,
            "sample": f"{nb} batches x {batch} queries ({dt:.1f} s), {n_docs} x {d} fp32 unit-norm corpus, k={k}; "
                      f"oracle restatement of SimpleRetriever.batch_retrieve (retriever.py:131-166), "
                      f"BLAS on {cores} threads (the cores granted to this process)",
            "batched_sgemm": {"value": round(batch * nb2 / dt2, 2), "unit": "queries/s", "batches": nb2,
                              "note": "not the reference algorithm: one Q @ A.T sgemm per batch + per-row "
                                      "argpartition/argsort (a stronger CPU point)"}}


def algorithmic_bytes(rows: int, d: int, batch: int, dtype: str, metric: str, screen16: bool = False,
                      screen8: bool = False) -> int:
    """HBM bytes one corpus-streaming launch must move: the rows once (4 B/element fp32 and fp32-split, 2 B bf16,
    2 B when the fp32 screen streams the f16 screening copy, 1 B the int8 copy), the per-row factors it reads (norm
    for cosine, row scale for fp32-split; the int8 copy's norm, scale and error norm), the queries once (fp32; the
    int8 screen's two int8 pieces of 32 slots, or bf16 storage's one piece of 64 slots) and their 4 scalars."""
    if screen8:
        slots = 64 if dtype == "bf16" and batch > 32 else 32
        return rows * (d + 12) + 64 * d + 4 * slots * 4
    elem = 2 if dtype == "bf16" or screen16 else 4
    # per-row factors: the norm (cosine; and the fp32 screen's error bound for either metric), the split scale
    per_row = (4 if metric == "cosine" or dtype == "fp32" else 0) + (4 if dtype == "fp32-split" else 0)
    return rows * (d * elem + per_row) + batch * d * 4


def make_stager(ix, q, nb: int, local: int, restage: bool, seed: int = 4242):
    """A step's queries: with `restage` (the default) every step stages a NEW batch of B queries already resident in HBM
    (nb distinct batches in one device buffer, batch 0 = q; rr_set_queries_device — the copy into the library's query
    buffer and the int8 screens' query pieces, on its staging stream), as a serving loop does per batch; without, the
    batch staged once is searched again (round 5's loop). Returns (stage(i) or None, keep-alive)."""
    if not restage:
        return None, None
    rng = np.random.default_rng(seed)
    qs = rng.standard_normal((nb,) + q.shape).astype(np.float32)
    qs /= np.linalg.norm(qs, axis=2, keepdims=True)
    qs[0] = q
    try:
        import torch
        dev = torch.from_numpy(qs).to(f"cuda:{local}")
        torch.cuda.synchronize()
        ptrs = [dev[i].data_ptr() for i in range(nb)]
        b, d = q.shape

        def stage(i):
            ix.set_queries_device(ptrs[i % nb], b, d)
        return stage, dev
    except Exception:   # (no torch: the pinned host path, rr_set_queries)
        def stage(i):
            ix.set_queries(qs[i % nb])
        return stage, qs


def timed_steps(ix, k, steps, warmup, dist, cuda_sync, every=1, acct=None, stage=None):
    """W untimed warmup steps, then exactly K steps between barrier + device sync on both sides.
    HIP events bracket the similarity kernel of every `every`-th step (event markers cost GPU time
    between kernels; sampling keeps the duration measurement inside the timed region).

    Screened searches (fp32 storage) whose bound could not prove the top-k are flagged on the device and owe an
    exact re-run; a staged search nobody fetches is superseded by the next one and never re-run by the library. So
    INSIDE the timed region, after the K steps, the flagged blocks of the window are counted (rr_screen_counts) and
    every one the library did not already re-run is paid for with one exact search (RR_KERNEL_EXACT) before the
    closing sync. Multi-process: the ranks' counts are summed (a block flagged on any rank is re-run by all; the
    sum may over-pay, never under-pay) and every rank runs that many exact searches (their all-gathers pair up).
    `acct` (dict, optional) receives {"flagged": F, "reruns_library": R, "reruns_paid": P, "blocks": B,
    "wide_slots": W} (W: query slots the verify proved in its wide phase, no re-run needed).
    Returns (wall seconds, fused-kernel event ms summed, fused launches timed)."""
    from rag_service_amd.dist import barrier, sum_over_ranks
    for i in range(warmup):
        if stage:
            stage(i)
        ix.search_staged(k)
    ix.synchronize()
    b0, f0, r0, w0 = ix.screen_counts_all()
    ix.set_timing(True)
    ix.kernel_time(reset=True)
    barrier(dist)
    cuda_sync()
    ix.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        if every > 1:
            ix.set_timing(i % every == 0)
        if stage:
            stage(warmup + i)
        ix.search_staged(k)
    t_enq = time.perf_counter() - t0           # host time to enqueue the K steps (the device may still be running)
    b1, f1, r1, w1 = ix.screen_counts_all()    # synchronises (and settles the last search)
    owed = int(sum_over_ranks(dist, float(max(0, (f1 - f0) - (r1 - r0)))))
    if owed:
        ix.set_timing(False)
        prev = ix.kernel
        ix.set_kernel("exact")
        for _ in range(owed):
            ix.search_staged(k)
        ix.set_kernel(prev)
    ix.synchronize()
    cuda_sync()
    barrier(dist)
    elapsed = time.perf_counter() - t0
    kern_ms, launches = ix.kernel_time(reset=True)
    ix.set_timing(False)
    if acct is not None:
        acct.update({"blocks": b1 - b0, "flagged": f1 - f0, "reruns_library": r1 - r0, "reruns_paid": owed,
                     "wide_slots": w1 - w0, "host_enqueue_ms_per_step": round(t_enq / max(steps, 1) * 1e3, 4)})
    return elapsed, kern_ms, launches


def clustered_field(args, local: int, cuda_sync, steps: int = 60, warmup: int = 80, sigma: float = 0.03) -> dict:
    """Data dependence of the screened search: the headline's search (k, cosine) over 1M-row corpora
    built from the reference's only real embeddings (data/squad_embeddings.npy, 1000 e5 rows, a committed fixture):
    row i = SQuAD row c(i) + seeded Gaussian noise of relative size sigma, L2-normalised — "interleaved" (c(i) = i mod
    1000) and "contiguous" (c(i) = i div (n / 1000): clusters stored in topic order, the normal case for an ingested
    corpus). Per layout, after `warmup` awaited searches (the adaptive screen settles): screened q/s over `steps` staged
    steps with every flagged block's exact re-run paid inside the window, the exact one-pass kernel's q/s, which copy
    screened, repair mode and the slots it completed, and whether a fetched result equals the exact kernel's bit for
    bit (tools/clustered_bench.py has the sigma sweep)."""
    from rag_service_amd import Index
    squad = np.load(os.path.join(REPO, "tests", "golden", "data", "squad_embeddings.npy")).astype(np.float32)
    squad /= np.linalg.norm(squad, axis=1, keepdims=True)
    n, d = args.docs, squad.shape[1]
    rng = np.random.default_rng(20260)
    noise = rng.standard_normal((n, d), dtype=np.float32) / np.float32(np.sqrt(d))
    qrng = np.random.default_rng(777)
    qc = qrng.integers(0, squad.shape[0], args.batch)
    q = squad[qc] + np.float32(sigma) * qrng.standard_normal((args.batch, d), dtype=np.float32) / np.float32(np.sqrt(d))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    out = {"sigma": sigma, "docs": n, "k": args.k, "steps": steps, "warmup_awaited": warmup,
           "source": "tests/golden/data/squad_embeddings.npy (the reference's data/squad_embeddings.npy)"}
    ix = Index(devices=[local], dtype="fp32", metric=args.metric)
    for layout in ("interleaved", "contiguous"):
        c = np.arange(n) % squad.shape[0] if layout == "interleaved" else np.minimum(np.arange(n) // (n // squad.shape[0]),
                                                                                       squad.shape[0] - 1)
        corpus = squad[c]
        corpus += np.float32(sigma) * noise
        corpus /= np.linalg.norm(corpus, axis=1, keepdims=True)
        ix.set_kernel("auto")
        ix.load(corpus)
        del corpus
        ix.set_queries(q)
        for _ in range(warmup):
            ix.search_staged(args.k)
            ix.synchronize()
        acct = {}
        s_el, _, _ = timed_steps(ix, args.k, steps, 0, None, cuda_sync, 10, acct)
        state = ix.screen_state()
        i8, repaired = ix.screen_int8(), ix.screen_repairs()
        got = ix.search(q, args.k)
        ix.set_kernel("exact")
        ix.set_queries(q)
        e_el, _, _ = timed_steps(ix, args.k, steps, 5, None, cuda_sync, 10)
        want = ix.search(q, args.k)
        out[layout] = {"screened_qps": round(args.batch * steps / s_el, 1),
                       "exact_qps": round(args.batch * steps / e_el, 1), "speedup_vs_exact": round(e_el / s_el, 3),
                       "screen_copy": "int8" if i8 else "f16", "repair_mode": bool(state[0]), "pauses": state[2],
                       "repaired_slots_since_load": repaired, "flagged_timed": acct["flagged"],
                       "reruns_paid_timed": acct["reruns_paid"],
                       "bit_identical_to_exact": bool(np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0]))}
    ix.close()
    del noise
    return out


def spawn_ranks(n: int) -> int:
    """Run this script under torch.distributed.run with one rank per GPU, as a child process (this process
    has not touched the GPU). Returns the child's exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp32-split"])
    ap.add_argument("--variants", default="bf16,fp32-split",
                    help="other corpus dtypes measured on the same workload (N=1 only; reported beside value)")
    ap.add_argument("--variant-steps", type=int, default=100)
    ap.add_argument("--metric", default="cosine", choices=["cosine", "dot"])
    ap.add_argument("--latency-steps", type=int, default=1000,
                    help="synchronous batches timed one by one for p50/p99 (BASELINE.md: >= 1000), and batches of the "
                         "pipelined host-inclusive loop")
    ap.add_argument("--timing-every", type=int, default=0,
                    help="bracket the similarity kernel with HIP events on every N-th timed step "
                         "(0: every 5th step when --steps < 100, else every 10th)")
    ap.add_argument("--steady-steps", type=int, default=2000,
                    help="back-to-back steps timed again after the latency loop (steady-state rate, reported "
                         "beside value; BASELINE.md: >= 1000 steps)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "exact", "fused"],
                    help="similarity kernel of the timed loops (rr_set_kernel; A/B and counter passes: `exact` = the "
                         "one-pass exact fp32 kernel without the screen)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-clustered", action="store_true",
                    help="skip the clustered-corpus field (two SQuAD-derived 1M-row corpora; N=1 only)")
    ap.add_argument("--exchange-1rank", action="store_true",
                    help="N=1: run the multi-GPU data path anyway (a 1-rank RCCL communicator: per-block all-gather "
                         "of the candidates and the device merge), for measuring the exchange's cost on one GPU")
    ap.add_argument("--ingest-rows", type=int, default=262_144,
                    help="rows of a host fp32 array timed through rr_load (N=1 only; 0 = skip)")
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of per-query CPU baseline work (at least one batch)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc FETCH_SIZE child pass that fills roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / control-plane check without a GPU: every rank joins the gloo group, "
                         "reaches the timed-loop barrier and rank 0 prints one JSON line")
    ap.add_argument("--dist-timeout-s", type=float, default=300.0,
                    help="N>1: deadline of every cross-rank wait — the gloo control plane's collectives and (a "
                         "third of it, at most 120 s) the library's waits on RCCL work; a miss ends the rank with a "
                         "JSON error line naming the rank and stage, and a non-zero exit status")
    ap.add_argument("--dry-run-stall-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--no-restage", action="store_true",
                    help="search the batch staged once in every step (round 5's loop) instead of staging a new batch, "
                         "resident in HBM, per step")
    ap.add_argument("--shard-group", type=int, default=0,
                    help="N>1: ranks per shard group S (the corpus as S row shards with one RCCL all-gather per block, "
                         "groups searching their own batches; R = N / S replica groups); 0 = auto: the fewest ranks "
                         "whose shards keep >= 500k rows (rag_service_amd.dist.placement); N = pure row shards")
    ap.add_argument("--no-row-shard-all", action="store_true",
                    help="with R > 1 replica groups, skip the second measurement over all N ranks as row shards")
    ap.add_argument("--idle-start", action="store_true",
                    help="prepare the step batches on the host after the corpus build (the round-5 order): the GPU idles "
                         "for that preparation right before the warm-up steps")
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)   # (test hook: every rank on cuda:0)
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a path setting of the measured handle (rr_set_option: screen_grid, verify_cus, x_slots, "
                         "x_host_wait_us, screen_i8_pieces, ...; results are the same under every value); repeatable")
    args = ap.parse_args()
    args.options = {}
    for o in args.opt:
        name, _, value = o.partition("=")
        args.options[name.strip()] = int(value)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    from rag_service_amd.dist import env_rank_world
    rank, world, _ = env_rank_world()
    # (No GPU_MAX_HW_QUEUES override: the library's streams take the runtime's high-priority queue pool, which RCCL's
    # internal streams never share at any queue count; DESIGN §5 "Hardware queues", profiles/r04/queues/.)
    stage = {"stage": "start"}
    try:
        run(args, stage)
    except Exception as e:   # a missed deadline (RCCL or gloo) or any failure: say which rank and where, exit != 0
        from rag_service_amd._lib import HipRetrievalError
        code = e.code if isinstance(e, HipRetrievalError) else None
        print(json.dumps({"metric": METRIC, "value": None, "error": f"{type(e).__name__}: {e}"[:600],
                          "error_code": code, "rank": rank, "n_gpus": world, "stage": stage["stage"]}), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        # no interpreter teardown: destructors would wait on device work that may never finish (a peer is gone)
        os._exit(3)


def run(args, stage: dict) -> None:
    # (HIP events on every 5th step of a short window: two event records per timed step are host work in the window)
    every = args.timing_every or (5 if args.steps < 100 else 10)

    from rag_service_amd import Index, get_unique_id
    from rag_service_amd import _lib
    from rag_service_amd.dist import (all_gather_bytes, barrier, broadcast_bytes, env_rank_world,
                                      init_control_plane, max_over_ranks, placement, sum_over_ranks)

    rank, world, local = env_rank_world()
    if args.same_device:
        local = 0
    # placement: R replica groups of S ranks; group g holds the whole corpus as S row shards (its own RCCL
    # communicator) and searches its own batches
    S, R = placement(args.docs, world, args.shard_group)
    grp, grank = rank // S, rank % S
    stage["stage"] = "control-plane init"
    dist = init_control_plane(world, rank, timeout_s=max(1, int(args.dist_timeout_s)))
    if args.dry_run:
        if rank == args.dry_run_stall_rank:   # (test hook: a rank that never reaches the barrier in time)
            time.sleep(args.dist_timeout_s + 3)
        stage["stage"] = "dry-run barrier"
        barrier(dist)
        ranks_seen = max_over_ranks(dist, float(rank)) + 1
        # the groups' communicator ids as the real run exchanges them (stand-in ids: no GPU call)
        ids = all_gather_bytes(dist, f"group-{grp}".encode() if grank == 0 else None)
        ids_ok = sum_over_ranks(dist, float(ids[grp * S] == f"group-{grp}".encode()))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": int(ranks_seen),
                              "launched_by": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ
                              else "plain",
                              "placement": {"shard_group": S, "replica_groups": R,
                                            "ranks_with_their_group_id": int(ids_ok)}}), flush=True)
        barrier(dist)
        return

    try:
        import torch
        torch.cuda.set_device(local)
        cuda_sync = torch.cuda.synchronize
    except Exception:  # torch is plumbing only: timing does not depend on it
        def cuda_sync():
            return None

    stage["stage"] = "handle + RCCL communicator"
    ix = Index(devices=[local], dtype=args.dtype, metric=args.metric, options=args.options)
    rccl_ranks = 0
    if S > 1:   # the group's communicator: its first rank's id, exchanged over the control plane
        uids = all_gather_bytes(dist, get_unique_id() if grank == 0 else None)
        ix.init_dist(S, grank, uids[grp * S])
        rccl_ranks = ix.dist_info()[0]
    elif args.exchange_1rank:
        ix.init_dist(1, 0, get_unique_id())
        rccl_ranks = ix.dist_info()[0]
    if S > 1:   # the library's waits on RCCL work: a third of the control-plane deadline, at most 120 s
        ix.set_timeout(int(min(120.0, args.dist_timeout_s / 3) * 1000))
    # the hardware queues the handle's four streams dispatch to (distinct = none shares an in-order queue)
    queues = ix.stream_queues(0)
    rng = np.random.default_rng(5678 + grp)   # (each replica group searches batches of its own)
    q = rng.standard_normal((args.batch, args.dim)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    # The host-side preparation of the step batches (NumPy, torch's first device copy) comes BEFORE the corpus build
    # unless --idle-start: the W warm-up and K timed steps then follow the build without the GPU idling for the ~5-10
    # ms that preparation takes (measured both ways: DESIGN §4, profiles/r06/idle_start/). No GPU work is added.
    if not args.idle_start:
        stager, _keep = make_stager(ix, q, 16, local, not args.no_restage, 4242 + grp)
    stage["stage"] = "corpus fill"
    ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, args.docs, args.dim)
    if args.kernel != "auto":
        ix.set_kernel(args.kernel)
    sb, se = ix.shard_range(0)

    # ---- throughput: queries resident in HBM, K back-to-back steps, each a new batch ---------------
    stage["stage"] = "timed steps"
    ix.set_queries(q)
    if args.idle_start:
        stager, _keep = make_stager(ix, q, 16, local, not args.no_restage, 4242 + grp)
    acct = {}
    elapsed, kern_ms, launches = timed_steps(ix, args.k, args.steps, args.warmup, dist, cuda_sync, every, acct,
                                             stager)
    elapsed = max_over_ranks(dist, elapsed)
    stage["stage"] = "latency loops"

    # ---- latency: host queries in -> host results out, one batch at a time ------------------------
    lat = []
    for i in range(args.latency_steps):
        barrier(dist)
        t = time.perf_counter()
        ix.search(q, args.k)
        lat.append(time.perf_counter() - t)
    lat_ms = np.array(lat) * 1e3
    p50 = max_over_ranks(dist, float(np.percentile(lat_ms, 50)))
    p99 = max_over_ranks(dist, float(np.percentile(lat_ms, 99)))
    _, head_idx = ix.search(q, args.k)

    # ---- pipelined host-inclusive rate: H2D + search + D2H of each batch enqueued asynchronously, two
    # batches in flight (rr_search_async / rr_wait), the cost the reference's batch_retrieve pays
    # (retriever.py:738,773) ---------------------------------------------------------------------------
    barrier(dist)
    t = time.perf_counter()
    tickets = []
    for i in range(args.latency_steps):
        tickets.append(ix.search_async(q, args.k))
        if len(tickets) == 2:
            ix.wait(tickets.pop(0))
    for tk in tickets:
        ix.wait(tk)
    host_pipe_s = max_over_ranks(dist, time.perf_counter() - t)

    # ---- steady state: the same staged loop again, long after the GPU left idle ---------------------
    stage["stage"] = "steady-state steps"
    st_acct = {}
    st_el, st_ms, st_n = timed_steps(ix, args.k, args.steady_steps, 0, dist, cuda_sync, 10, st_acct, stager)
    st_el = max_over_ranks(dist, st_el)
    scr_blocks, scr_fallbacks = ix.screen_stats()
    stage["stage"] = "single-stream and exact-kernel loops"

    # ---- roofline of the fused kernel (rank 0's shard) ---------------------------------------------
    n_local = se - sb
    # the fp32 screened search (k <= 29) streams the f16 screening copy when the handle keeps one
    screen16 = args.dtype == "fp32" and args.k <= 29 and args.kernel == "auto" and ix.screen_copy()
    # bf16 storage screens its int8 copy (DT 9): 32-slot blocks (batch <= 32, k <= 29) and 64-slot ones (16-entry
    # lists: k <= 13)
    screen_bf = (args.dtype == "bf16" and args.k <= (13 if args.batch > 32 else 29) and args.kernel == "auto" and
                 ix.screen_int8())
    screen8 = (screen16 and ix.screen_int8()) or screen_bf   # the int8 copy, unless the adaptive screen gave it up
    alg_bytes = algorithmic_bytes(n_local, args.dim, args.batch, args.dtype, args.metric, screen16, screen8)
    fp32_floor = n_local * args.dim * 4 + args.batch * args.dim * 4
    avg_kernel_s = (kern_ms / max(launches, 1)) / 1e3
    step_s = elapsed / args.steps
    # screened blocks on two compute streams (the fp32 default): block i + 1's screen starts while block i's screen
    # drains and its verify runs, so each launch's event span covers about two steps and is no duration of its
    # own. One launch per step: the launch's time is then the step time, and `achieved` = its algorithmic bytes /
    # ms_per_step (the sustained HBM rate of the path). The kernel alone (one stream, every CU) is measured below.
    streams = ix.compute_streams() if args.dtype == "fp32" or screen_bf else 1
    overlap = streams == 2
    launch_s = step_s if overlap else avg_kernel_s
    achieved = alg_bytes / launch_s / 1e9 if launches else None
    consistent = bool(launches) and launch_s <= step_s * 1.001
    st_launch_s = (st_el / args.steady_steps) if overlap else (st_ms / max(st_n, 1) / 1e3)
    alone = None
    if overlap and not args.pmc_child:
        # the same screen kernel with one compute stream (every CU screening, nothing overlapping): its own launch
        # duration by HIP events on every launch, after the GPU has been busy for the loops above
        ix.compute_streams(1)
        a_el, a_ms, a_n = timed_steps(ix, args.k, 40, 5, dist, cuda_sync, 1, None, stager)
        ix.compute_streams(2)
        a_kern = a_ms / max(a_n, 1) / 1e3
        alone = {"kernel_avg_us": round(a_kern * 1e6, 2), "frac": round(alg_bytes / a_kern / 1e9 / HBM_PEAK_GBS, 4),
                 "ms_per_step": round(a_el / 40 * 1e3, 4), "launches": a_n,
                 "note": "compute_streams(1): the screen on every CU, one launch at a time, 40 steps after the loops "
                         "above; HIP events around every launch"}
    if args.pmc_child:            # only the fused-kernel launches matter to the parent's PMC parse
        ix.close()
        return

    # ---- replica groups (R > 1): the same workload with all N ranks as ONE row-sharded group (the north star's
    # layout, one RCCL all-gather over all N per block), reported beside value ----------------------------------
    row_all = None
    if R > 1 and not args.no_row_shard_all:
        stage["stage"] = "all ranks as one row-sharded group"
        ix.close()
        ax = Index(devices=[local], dtype=args.dtype, metric=args.metric, options=args.options)
        ax.init_dist(world, rank, broadcast_bytes(dist, get_unique_id() if rank == 0 else None))
        ax.set_timeout(int(min(120.0, args.dist_timeout_s / 3) * 1000))
        ax.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, args.docs, args.dim)
        q0 = np.random.default_rng(5678).standard_normal((args.batch, args.dim)).astype(np.float32)
        q0 /= np.linalg.norm(q0, axis=1, keepdims=True)
        ax.set_queries(q0)
        a_stager, _akeep = make_stager(ax, q0, 16, local, not args.no_restage)
        a_acct, a_st = {}, {}
        aw_el, _, _ = timed_steps(ax, args.k, args.steps, args.warmup, dist, cuda_sync, every, a_acct, a_stager)
        aw_el = max_over_ranks(dist, aw_el)
        as_el, _, _ = timed_steps(ax, args.k, args.steady_steps, 0, dist, cuda_sync, 10, a_st, a_stager)
        as_el = max_over_ranks(dist, as_el)
        row_all = {"value": round(args.batch * args.steps / aw_el, 2), "unit": "queries/s",
                   "ms_per_step": round(aw_el / args.steps * 1e3, 4),
                   "steady_value": round(args.batch * args.steady_steps / as_el, 2),
                   "steady_ms_per_step": round(as_el / args.steady_steps * 1e3, 4),
                   "parallelism": f"row-shard x{world}", "rccl_ranks": ax.dist_info()[0],
                   "screen_fallbacks_timed": a_acct.get("flagged"), "reruns_paid": a_acct.get("reruns_paid"),
                   "note": "the same K / W staged loop and steady loop with all N ranks as one group: every rank "
                           "searches every batch over its 1/N row shard, one RCCL all-gather over all N per block"}
        ax.close()

    # ---- the other corpus dtypes on the same workload (1 GPU only; reported beside, never `value`) --
    # ---- corpus ingest (main.py:20-23 + retriever.py:582): host fp32 numpy -> HBM storage, N=1 only ------
    ingest = None
    if world == 1 and args.ingest_rows > 0:
        host = np.full((args.ingest_rows, args.dim), 0.03125, dtype=np.float32)   # pages touched
        lx = Index(devices=[local], dtype=args.dtype, metric=args.metric)
        lx.load(host[: min(1024, args.ingest_rows)])                                 # warm the path
        t = time.perf_counter()
        lx.load(host)
        t_load = time.perf_counter() - t
        lx.close()
        ingest = {"GBps": round(host.nbytes / t_load / 1e9, 2), "rows": args.ingest_rows,
                  "seconds": round(t_load, 4),
                  "note": "rr_load of a pageable host fp32 array: 2 pinned 32 MiB staging buffers, threaded host "
                          "copy overlapped with H2D DMA + on-device layout/dtype conversion and norms"}
        del host

    variants = {}
    if world == 1 and (args.dtype == "fp32" or screen_bf) and args.variant_steps > 0 and args.kernel == "auto":
        # the one-pass exact fp32 kernel (RR_KERNEL_EXACT, DT 3) on the same handle: it streams the fp32 rows the
        # reference streams (retriever.py:600), and it is what a flagged block's re-run and any corpus the screen
        # cannot prune cost
        ix.set_kernel("exact")
        e_el, e_ms, e_n = timed_steps(ix, args.k, args.variant_steps, args.warmup, dist, cuda_sync, 10, None, stager)
        _, e_idx = ix.search(q, args.k)
        ix.set_kernel("auto")
        e_kern = e_ms / max(e_n, 1) / 1e3
        e_ach = algorithmic_bytes(n_local, args.dim, args.batch, args.dtype, args.metric) / e_kern / 1e9
        variants["exact_" + args.dtype] = {
            "value": round(args.batch * args.variant_steps / e_el, 2), "unit": "queries/s",
            "ms_per_step": round(e_el / args.variant_steps * 1e3, 4), "kernel_avg_us": round(e_kern * 1e6, 2),
            "achieved_GBps": round(e_ach, 1), "frac": round(e_ach / HBM_PEAK_GBS, 4), "steps": args.variant_steps,
            "alg_bytes_per_launch": algorithmic_bytes(n_local, args.dim, args.batch, args.dtype, args.metric),
            "index_agreement_with_headline": round(float(np.mean(e_idx == head_idx)), 4),
            "note": ("RR_KERNEL_EXACT: sk_score_kernel DT 3 (fp32 rows, each value split exactly into 3 bf16, 6 bf16 "
                     "MFMAs) over the fp32 rows, one pass, no screen; HIP events on every 10th launch"
                     if args.dtype == "fp32" else
                     "RR_KERNEL_EXACT: sk_score_kernel DT 1 over the bf16 rows (64 query slots, bf16 hi + lo query "
                     "pieces), one pass, no screen; HIP events on every 10th launch")}
    if world == 1 and args.variants:
        for vd in [v for v in args.variants.split(",") if v and v != args.dtype]:
            vx = Index(devices=[local], dtype=vd, metric=args.metric)
            vx.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, args.docs, args.dim)
            vx.set_queries(q)
            v_stager, _vkeep = make_stager(vx, q, 16, local, not args.no_restage)
            v_acct = {}
            v_el, v_ms, v_n = timed_steps(vx, args.k, args.variant_steps, args.warmup, dist, cuda_sync, 10, v_acct,
                                          v_stager)
            _, v_idx = vx.search(q, args.k)
            # bf16 storage screens its int8 copy (DT 9, verified by the bf16 pass's own arithmetic): the screen streams
            # that copy, so its bytes are the launch's algorithmic bytes; the screened steps overlap on two streams
            v_scr = vd == "bf16" and args.k <= (13 if args.batch > 32 else 29) and vx.screen_int8()
            v_bytes = algorithmic_bytes(n_local, args.dim, args.batch, vd, args.metric, screen8=v_scr)
            vx.close()
            v_kern = v_ms / max(v_n, 1) / 1e3
            v_step = v_el / args.variant_steps
            v_ach = v_bytes / (v_step if v_scr else v_kern) / 1e9
            variants[vd] = {"value": round(args.batch * args.variant_steps / v_el, 2), "unit": "queries/s",
                            "ms_per_step": round(v_step * 1e3, 4),
                            "kernel_avg_us": round(v_kern * 1e6, 2), "achieved_GBps": round(v_ach, 1),
                            "frac": round(v_ach / HBM_PEAK_GBS, 4), "steps": args.variant_steps,
                            "alg_bytes_per_launch": v_bytes, "screened": bool(v_scr),
                            "screen_fallbacks_timed": v_acct.get("flagged"), "reruns_paid": v_acct.get("reruns_paid"),
                            "index_agreement_with_headline": round(float(np.mean(v_idx == head_idx)), 4)}
            if v_scr:
                variants[vd]["note"] = ("the screened search over the int8 copy of the bf16 rows (DT 9, one query piece), "
                                        "verified by the bf16 pass's own arithmetic; frac = its bytes / step time (two "
                                        "compute streams overlap the launches), every flagged block's exact re-run paid")

    clustered = None
    if world == 1 and args.dtype == "fp32" and not args.no_clustered and args.variants:
        stage["stage"] = "clustered corpora"
        try:
            clustered = clustered_field(args, local, cuda_sync)
        except Exception as e:   # reported, never fatal to the headline line
            clustered = {"error": f"{type(e).__name__}: {e}"[:300]}
    traffic, traffic_note, mfma = None, "not measured", None
    if rank == 0 and world == 1 and not args.no_pmc:
        ix.close()                 # free HBM for the child pass
        traffic, traffic_note, mfma = pmc_counters(args, alone["kernel_avg_us"] / 1e6 if alone else avg_kernel_s)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:   # rank 0 at N=1 only
            cpu = cpu_baseline(args.docs, args.dim, args.batch, args.k, args.cpu_budget)
        value = args.batch * args.steps * R / elapsed   # (R replica groups, each its own batches)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if R == 1 else "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (device-generated unit-norm approx-Gaussian rows, seed 1234; unit-norm queries)",
            "config": {"workload": f"{args.docs} synthetic docs d={args.dim}, batch={args.batch}, top-k={args.k}, "
                                   f"{args.metric} (CupyRetriever semantics)",
                       "docs": args.docs, "d": args.dim, "batch": args.batch, "k": args.k,
                       "metric": args.metric, "corpus_dtype": args.dtype,
                       "parallelism": f"row-shard x{S}" + (f", replica groups x{R}" if R > 1 else "")},
            "placement": {"shard_group": S, "replica_groups": R, "rule": (
                "auto: the fewest ranks whose row shards keep >= 500k rows each (rag_service_amd.dist.placement)"
                if args.shard_group == 0 else f"--shard-group {args.shard_group}"),
                "note": "each group holds the whole corpus as S contiguous row shards and searches its own batches "
                        "(one RCCL all-gather over its S ranks per block); value = the R groups' batches together "
                        "over the max-over-ranks time"},
            "row_shard_all": row_all,
            "p50_ms": round(p50, 4),
            "p99_ms": round(p99, 4),
            "latency_note": "host-inclusive per batch: H2D queries + pipeline + D2H results, synchronous",
            "setup_order": ("--idle-start: the step batches prepared on the host after the corpus build (the GPU idle "
                            "for that right before the W warm-up steps)" if args.idle_start else
                            "the step batches prepared on the host before the corpus build, so the W warm-up and K timed "
                            "steps follow the build without an idle gap (no GPU work added; --idle-start gives the other "
                            "order: profiles/r06/idle_start/)"),
            "step_queries": ("every step stages a new batch resident in HBM (16 distinct unit-norm batches, "
                             "rr_set_queries_device: the copy into the library's query buffer and the int8 screens' "
                             "query pieces, on its staging stream)" if not args.no_restage else
                             "the batch staged once, searched in every step"),
            "host_pipelined": {"value": round(args.batch * args.latency_steps * R / host_pipe_s, 2),
                               "unit": "queries/s",
                               "batches": args.latency_steps, "in_flight": 2,
                               "note": "host numpy queries in, host results out: rr_search_async (pinned H2D + "
                                       "search + D2H enqueued) / rr_wait, two batches in flight"},
            "host_enqueue_ms_per_step": {"window": acct.get("host_enqueue_ms_per_step"),
                                         "steady": st_acct.get("host_enqueue_ms_per_step"),
                                         "note": "host time to enqueue one search step (rr_search_staged) in the timed "
                                                 "loops: below ms_per_step, the device and not the host sets the rate"},
            "steady_state": {"value": round(args.batch * args.steady_steps * R / st_el, 2), "unit": "queries/s",
                             "steps": args.steady_steps,
                             "ms_per_step": round(st_el / args.steady_steps * 1e3, 4),
                             "kernel_avg_us": round(st_ms / max(st_n, 1) * 1e3, 2),
                             "frac": round(alg_bytes / st_launch_s / 1e9 / HBM_PEAK_GBS, 4) if st_n else None,
                             "note": "the same staged loop after the latency loops (GPU long out of idle); "
                                     "value above is the first K steps after W warm-up steps from idle"},
            "exchange": ("rccl ncclAllGather of per-shard top-k keys, device merge on every rank"
                         if S > 1 or rccl_ranks else "none (one shard)"),
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default (4)"),
            "library_build": _lib.build_info(),
            "options": args.options,
            "rr_env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("RR_")},
            "stream_queues_distinct": len(set(v for v in queues if v)),
            "stream_priority_range": stream_priority_range(),
            "rccl_ranks": rccl_ranks,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic,
                         "traffic_note": traffic_note,
                         "mfma": mfma,
                         "kernel": SCORE_KERNEL_DOC,
                         "kernel_avg_us": round(launch_s * 1e6, 2),
                         "kernel_span_us": round(avg_kernel_s * 1e6, 2),
                         "kernel_alone": alone,
                         "kernel_timing": (f"HIP events on the kernel's stream around every {every}-th "
                                           f"similarity-kernel launch of the timed region ({launches} launches)"
                                           + ("; two compute streams: consecutive launches overlap, kernel_span_us is "
                                              "a launch's event span, kernel_avg_us and achieved use the step time "
                                              "(one launch per step); kernel_alone is the kernel by itself"
                                              if overlap else "")),
                         "kernel_le_step": consistent,
                         "compute_streams": streams,
                         "step_frac": round(alg_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
                         "step_frac_note": "algorithmic bytes of one launch / ms_per_step: the sustained fraction of "
                                           "peak over the timed steps (with two compute streams the launches overlap "
                                           "and a launch's own span overstates its time)",
                         "alg_bytes_per_launch": alg_bytes,
                         # §8(d)'s basis: the fp32 rows the reference streams (N·D·4 + the queries), per step
                         "fp32_floor_bytes": fp32_floor,
                         "frac_vs_fp32_floor": round(fp32_floor / step_s / 1e9 / HBM_PEAK_GBS, 4),
                         "frac_vs_fp32_floor_steady": round(fp32_floor / (st_el / args.steady_steps) / 1e9
                                                            / HBM_PEAK_GBS, 4),
                         "basis_note": ("frac = the bytes the launch streams (the int8 or f16 screening copy + per-row "
                                        "factors) / step "
                                        "time; frac_vs_fp32_floor = the fp32 corpus bytes SURVEY §8(d) prices (4 B per "
                                        "element) / step time — above 1 because the screen proves most fp32 rows "
                                        "need not be read; valid only with every flagged block's exact re-run paid "
                                        "(screen_fallbacks_timed, reruns_paid)" if screen16 else
                                        "frac and frac_vs_fp32_floor on the same rows"),
                         "screen_copy": bool(screen16),
                         "screen_int8": bool(screen8),
                         "screen_fallbacks_timed": acct.get("flagged"),
                         "reruns_paid": acct.get("reruns_paid"),
                         "reruns_by_library_timed": acct.get("reruns_library"),
                         "wide_verified_slots_timed": acct.get("wide_slots"),
                         "screen_fallbacks_steady": st_acct.get("flagged"),
                         "reruns_paid_steady": st_acct.get("reruns_paid"),
                         "fallback_note": "blocks whose bound could not prove the top-k inside the timed window; each "
                                          "not already re-run by the library is paid with one exact search inside "
                                          "the window (bench.py timed_steps)",
                         "screened_blocks": scr_blocks, "screen_fallbacks": scr_fallbacks},
            "cpu_baseline": cpu,
            "clustered": clustered,
            "other_dtypes": variants or None,
            "ingest": ingest,
            "dtype_note": {"fp32": "fp32 rows stored exactly; split-K kernel splits corpus and query values exactly "
                                   "into 3 bf16 each, 6 bf16 MFMAs (every kept product exact, dropped terms "
                                   "< 2^-23 |xq|), fp32 accumulate",
                           "bf16": "bf16 rows (RNE), bf16 MFMA, fp32 accumulate",
                           "fp32-split": "fp32 rows as f16 hi+lo with per-row 2^e scale (22-bit significand), "
                                         "3 f16 MFMAs, fp32 accumulate"},
        }
        print(json.dumps(out), flush=True)
    barrier(dist)
    ix.close()


def pmc_counters(args, kernel_s):
    """One rocprofv3 --pmc pass (FETCH_SIZE, SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE: 3 of 4 TCC, 1 of 8 SQ,
    1 of 2 GRBM slots) over a short run of this same workload, as a CHILD process. Per similarity-kernel
    launch (median):
      traffic   = FETCH_SIZE * 1024 * 2 bytes (KiB; gfx950 reports half of a wide stream, MI355X_MICROARCH.md §HBM)
      mfma.busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x kernel cycles), kernel cycles =
                  GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) — the matrix-core duty cycle;
      mfma.alg_tflops = the metric's own flops (2·B·N·D) / the timed kernel duration, against the dense
                  peak of the dtype the products run on."""
    import csv
    import shutil
    import statistics
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found", None
    out = tempfile.mkdtemp(prefix="bench_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [exe, "--pmc", "FETCH_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "--output-format", "csv",
           "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "3", "--warmup", "1",
           "--latency-steps", "1", "--no-cpu-baseline", "--docs", str(args.docs), "--dim", str(args.dim),
           "--batch", str(args.batch), "--k", str(args.k), "--dtype", args.dtype, "--metric", args.metric,
           "--variants", "", "--kernel", args.kernel] + [a for o in args.opt for a in ("--opt", o)] + \
          (["--no-restage"] if args.no_restage else [])
    try:
        subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        vals = {}
        for root, _, files in os.walk(out):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for row in csv.DictReader(open(os.path.join(root, f))):
                        if is_score_kernel(row["Kernel_Name"]):
                            key = (row.get("Dispatch_Id", ""), row["Counter_Name"])
                            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
        per = {}
        for (_, name), v in vals.items():
            per.setdefault(name, []).append(v)
        if "FETCH_SIZE" not in per:
            return None, "no similarity-kernel FETCH_SIZE rows", None
        traffic = round(statistics.median(per["FETCH_SIZE"]) * 1024 * 2)
        note = (f"rocprofv3 --pmc child pass, median of {len(per['FETCH_SIZE'])} similarity-kernel launches, "
                f"FETCH_SIZE x1024 B/KiB x2 (gfx950)")
        mfma = None
        if "SQ_VALU_MFMA_BUSY_CYCLES" in per and "GRBM_GUI_ACTIVE" in per:
            import torch
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            busy = statistics.median(per["SQ_VALU_MFMA_BUSY_CYCLES"])
            cyc = statistics.median(per["GRBM_GUI_ACTIVE"]) / 8
            flops = 2.0 * args.batch * args.docs * args.dim
            peak = {"fp32": 2500.0, "bf16": 2500.0, "fp32-split": 2500.0}[args.dtype]   # products on f16/bf16 MFMAs
            mfma = {"busy_frac": round(busy / (4 * cus * cyc), 4), "busy_cycles": busy, "kernel_cycles": cyc,
                    "clock_GHz": round(cyc / kernel_s / 1e9, 3) if kernel_s else None,
                    "alg_tflops": round(flops / kernel_s / 1e12, 2) if kernel_s else None,
                    "peak_tflops_dense": peak,
                    "note": "busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 x CUs x GRBM_GUI_ACTIVE/8); alg_tflops counts "
                            "2*B*N*D (the split-product MFMAs do 2-6x that on the matrix cores)"}
        return traffic, note, mfma
    except Exception as e:  # never fail the benchmark on the profiler
        return None, f"pmc pass failed: {type(e).__name__}", None
    finally:
        shutil.rmtree(out, ignore_errors=True)


if __name__ == "__main__":
    main()
