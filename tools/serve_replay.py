#!/usr/bin/env python3
"""Serving-level p50/p95/p99: replays the reference load test's request traces
(benchmarks/load_generator.py generate_trace; load_test.sh's "uniform" and "random" patterns, seed 10 +
offset) in-process through the reference's batching rule (RequestQueue.get_batch: up to 32 requests or a
1.0 s window, config.py:8-9) into BatchProcessor + HipRetriever, and prints the reference collector's
metrics (collector.py:34-69) as one JSON line per (pattern, rps).

    python tools/serve_replay.py [--rps 50,200,1000,4000] [--duration 10] [--rows 1000000]
                                 [--encoder table|e5] [--dtype fp32]

Queries: the 1000 real SQuAD questions (tests/golden/data/squad_queries.json), k = 2 (the HTTP default).
--encoder table: retrieval-only serving — each question's embedding is a fixed seeded unit-norm vector
  held on the GPU (no encoder cost), so the latency is batching + retrieval;
--encoder e5: the e5-large-shaped random-weight encoder of tools/bench_e2e.py (timing-faithful, parity
  unpinned) runs the embedding half on the GPU first.
The corpus is the headline's: --rows synthetic unit-norm rows x 1024 fp32. The LLM step is out of scope;
its stand-in echoes the prompt. Latency runs from a request's release to its stored result;
`client_poll` adds the reference client's 0.3 s polling quantisation (load_generator.py:91-116).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rag-serving-system_amd"), os.path.join(REPO, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rps", default="50,200,1000,4000")
    ap.add_argument("--duration", type=int, default=10)
    ap.add_argument("--patterns", default="uniform,random")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp32-split"])
    ap.add_argument("--encoder", default="table", choices=["table", "e5"])
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--max-wait", type=float, default=1.0)
    ap.add_argument("--k", type=int, default=2)
    args = ap.parse_args()

    import torch
    torch.cuda.is_available()
    from rag_service_amd import Index
    from rag_service_amd.core.batch_processor import BatchProcessor
    from rag_service_amd.core.retriever import HipRetriever
    from rag_service_amd.serving import EmbeddingTable, generate_trace, replay

    texts = json.load(open(os.path.join(REPO, "tests", "golden", "data", "squad_queries.json")))
    dev = "cuda:0"
    if args.encoder == "table":
        rng = np.random.default_rng(4321)
        table = rng.standard_normal((len(texts), 1024)).astype(np.float32)
        table /= np.linalg.norm(table, axis=1, keepdims=True)
        emb_model = EmbeddingTable(texts, table, dev).model
    else:
        from bench_e2e import WordHashTokenizer
        from transformers import XLMRobertaConfig, XLMRobertaModel
        torch.manual_seed(0)
        cfg = XLMRobertaConfig(vocab_size=250002, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                               intermediate_size=4096, max_position_embeddings=514, type_vocab_size=1,
                               pad_token_id=1, bos_token_id=0, eos_token_id=2, layer_norm_eps=1e-5)
        emb_model = {"tokenizer": WordHashTokenizer(),
                     "model": XLMRobertaModel(cfg, add_pooling_layer=False).eval()}

    # corpus generated on the device (bit-identical to the host generator), documents = row ids
    retr = HipRetriever(np.zeros((1, 1024), np.float32), ["0"], dtype=args.dtype)
    retr.index.fill_synthetic(1, 1234, args.rows, 1024)
    retr.N_A = args.rows
    retr.documents = [str(i) for i in range(args.rows)]
    seeds = {"uniform": 10, "random": 210, "poisson": 410}      # load_test.sh BASE_SEED + pattern offset
    with torch.no_grad():
        replay(BatchProcessor, retr, emb_model, texts, generate_trace("uniform", 64, 1, 0), k=args.k,
               max_batch_size=args.max_batch, max_wait_time=args.max_wait, device=dev)      # warm-up
        for pattern in args.patterns.split(","):
            for rps in (int(r) for r in args.rps.split(",")):
                trace = generate_trace(pattern, rps, args.duration, seeds[pattern])
                t0 = time.perf_counter()
                out = replay(BatchProcessor, retr, emb_model, texts, trace, k=args.k,
                             max_batch_size=args.max_batch, max_wait_time=args.max_wait, device=dev,
                             timeout=args.duration * 10 + 60)
                out.update({"pattern": pattern, "rps": rps, "duration_s": args.duration,
                            "seed": seeds[pattern], "rows": args.rows, "dtype": args.dtype,
                            "encoder": args.encoder, "max_batch": args.max_batch, "max_wait_s": args.max_wait,
                            "k": args.k, "wall_s": round(time.perf_counter() - t0, 2)})
                print(json.dumps(out), flush=True)
    retr.close()


if __name__ == "__main__":
    main()
