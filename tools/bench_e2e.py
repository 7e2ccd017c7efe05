#!/usr/bin/env python3
"""BASELINE config 4 — SQuAD end to end on one GPU: e5-large-shaped query encoder (PyTorch-ROCm) + the HIP
retriever, batch 32. Reports the latency split embed / retrieve.

    python tools/bench_e2e.py [--batches 30] [--warmup 3] [--batch 32] [--dtype fp32]

What runs is the reference's embedding half (batch_processor.py:81-92, restated in
rag_service_amd.core.batch_processor.embed_queries: "query: " prefix, padding + truncation, encoder forward,
last_hidden_state.mean(dim=1) over all positions, no L2 norm) followed by retrieval over the SQuAD corpus
(data/squad_embeddings.npy, 1000 x 1024) through HipRetriever — once with the query embeddings handed over
on the device (rr_set_queries_device) and once through the reference's host round trip (.cpu().numpy(),
batch_processor.py:92).

Not available offline, so stood in (timing-faithful, parity unpinned): the intfloat/multilingual-e5-large-
instruct weights (an XLM-RoBERTa-large architecture — 24 layers, hidden 1024, 16 heads, FFN 4096, vocab
250002 — randomly initialised, fp32 as the reference runs it) and its sentencepiece tokenizer (a word-hash
tokenizer with <s>/</s>/<pad> ids and ~1.3 pieces per word, the XLM-R average on these questions).
Queries: the 1000 real SQuAD questions (data/squad_queries.json), in batches of 32.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rag-serving-system_amd")]


class WordHashTokenizer:
    """Stand-in for the XLM-R sentencepiece tokenizer: <s>=0, <pad>=1, </s>=2; words of 7+ characters
    become two pieces. Right padding to the longest sequence, truncation to 512 (batch_processor.py:84-86)."""

    def __init__(self, vocab=250002, max_len=512):
        self.vocab, self.max_len = vocab, max_len

    def _ids(self, text):
        out = [0]
        for w in text.split():
            pieces = [w[: len(w) // 2], w[len(w) // 2:]] if len(w) >= 7 else [w]
            out += [5 + zlib.crc32(p.encode()) % (self.vocab - 5) for p in pieces]
        return (out[: self.max_len - 1] + [2])

    def __call__(self, texts, padding=True, truncation=True, return_tensors="pt"):
        import torch
        ids = [self._ids(t) for t in texts]
        L = max(len(x) for x in ids)
        return {"input_ids": torch.tensor([x + [1] * (L - len(x)) for x in ids]),
                "attention_mask": torch.tensor([[1] * len(x) + [0] * (L - len(x)) for x in ids])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--k", type=int, default=2, help="the HTTP default k (api/models.py:6)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "fp32-split"])
    args = ap.parse_args()

    import torch
    from transformers import XLMRobertaConfig, XLMRobertaModel
    from rag_service_amd.core.batch_processor import embed_queries
    from rag_service_amd.core.retriever import HipRetriever

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = XLMRobertaConfig(vocab_size=250002, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                           intermediate_size=4096, max_position_embeddings=514, type_vocab_size=1,
                           pad_token_id=1, bos_token_id=0, eos_token_id=2, layer_norm_eps=1e-5)
    model = XLMRobertaModel(cfg, add_pooling_layer=False).eval().to(dev)
    emb_model = {"tokenizer": WordHashTokenizer(), "model": model}

    corpus = np.load(os.path.join(REPO, "tests", "golden", "data", "squad_embeddings.npy"))
    queries = json.load(open(os.path.join(REPO, "tests", "golden", "data", "squad_queries.json")))
    retr = HipRetriever(corpus, list(range(corpus.shape[0])), dtype=args.dtype)

    def one_batch(i, handoff):
        qs = [queries[(i * args.batch + j) % len(queries)] for j in range(args.batch)]
        ks = [args.k] * args.batch
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        emb = embed_queries(emb_model, qs, dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if handoff:
            e = emb.float().contiguous()
            docs = retr.batch_retrieve_device(e.data_ptr(), e.shape[0], e.shape[1], ks)
        else:
            docs = retr.batch_retrieve(emb.cpu().numpy(), ks)
        t2 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, docs

    with torch.no_grad():
        for i in range(args.warmup):
            one_batch(i, True)
            one_batch(i, False)
        res = {}
        for handoff in (True, False):
            emb_ms, ret_ms, agree = [], [], []
            t0 = time.perf_counter()
            for i in range(args.batches):
                a, b, docs = one_batch(i, handoff)
                emb_ms.append(a)
                ret_ms.append(b)
            wall = time.perf_counter() - t0
            res["device_handoff" if handoff else "host_roundtrip"] = {
                "queries_per_s": round(args.batch * args.batches / wall, 2),
                "embed_ms_p50": round(float(np.percentile(emb_ms, 50)), 3),
                "embed_ms_p99": round(float(np.percentile(emb_ms, 99)), 3),
                "retrieve_ms_p50": round(float(np.percentile(ret_ms, 50)), 4),
                "retrieve_ms_p99": round(float(np.percentile(ret_ms, 99)), 4),
                "e2e_ms_p50": round(float(np.percentile(np.add(emb_ms, ret_ms), 50)), 3),
                "e2e_ms_p99": round(float(np.percentile(np.add(emb_ms, ret_ms), 99)), 3)}
        # the two hand-off forms return the same documents
        same = all(one_batch(i, True)[2] == one_batch(i, False)[2] for i in range(3))
    print(json.dumps({"config": "squad-e2e (BASELINE configs[3])", "batch": args.batch, "k": args.k,
                      "batches": args.batches, "corpus": list(corpus.shape), "corpus_dtype": args.dtype,
                      "encoder": "XLM-RoBERTa-large architecture (e5-large-instruct), random init, fp32",
                      "tokenizer": "word-hash stand-in (no sentencepiece model offline)",
                      "handoff_results_identical": same, **res}), flush=True)
    retr.close()


if __name__ == "__main__":
    main()
