"""Golden vectors for the embedding half, from the REFERENCE's BatchProcessor._process_batch itself
(rag_service/core/batch_processor.py:74-125; build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_embed_golden.py [short_facts|squad]

The reference runs on CPU with the deterministic stand-in models of tests/embed_fixture.py, its own
in-memory RequestQueue and its own CupyRetriever over the short_facts corpus (or the SQuAD corpus,
BASELINE config 4's: data/squad_embeddings.npy + squad_contexts.json, with the SQuAD questions) (NumPy
stand-in for the module-level cupy import, as make_golden.py). A wrapper around the retriever records the
(B, 1024) array _process_batch hands to batch_retrieve; the LLM stand-in records the prompts. Output
tests/golden/golden_embed[_squad].npz (embeddings per batch) + golden_embed[_squad].json (ks, documents,
prompts, stored results) — data only. `redis` gets an inert stand-in (only RedisRequestQueue touches it).
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(REPO, "tests"), HERE]

import embed_fixture as fx  # noqa: E402
from make_golden import import_reference, REF  # noqa: E402


def main(corpus_name="short_facts"):
    rd = types.ModuleType("redis")
    rd.from_url = lambda *a, **k: None
    sys.modules.setdefault("redis", rd)
    ret = import_reference()                      # cupy stand-in + /root/reference on sys.path
    import importlib
    bp = importlib.import_module("rag_service.core.batch_processor")
    rq = importlib.import_module("rag_service.core.request_queue")
    corpus = np.load(os.path.join(HERE, "data", f"{corpus_name}_embeddings.npy"))
    contexts = json.load(open(os.path.join(HERE, "data", f"{corpus_name}_contexts.json")))
    queries = json.load(open(os.path.join(HERE, "data", f"{corpus_name}_queries.json")))

    seen = []

    class Capture:
        def __init__(self, inner):
            self.inner = inner

        def batch_retrieve(self, q, ks):
            seen.append((np.array(q, copy=True), list(ks)))
            docs = self.inner.batch_retrieve(q, ks)
            seen[-1] += (docs,)
            return docs

    llm = fx.EchoLLM()
    queue = rq.RequestQueue()
    proc = bp.BatchProcessor(request_queue=queue, embedding_model={"tokenizer": fx.HashTokenizer(),
                                                                   "model": fx.make_encoder()},
                             llm_model=llm, retriever=Capture(ret.CupyRetriever(corpus, contexts)), device="cpu")
    out_npz, out_json = {}, {"batches": []}
    for bi, batch in enumerate(fx.batches(queries)):
        proc._process_batch(batch)
        emb, ks, docs = seen[bi]
        out_npz[f"emb{bi}"] = emb.astype(np.float32)
        out_json["batches"].append({"ks": ks, "docs": docs, "prompts": llm.prompts[bi],
                                    "results": {r["id"]: queue.results[r["id"]] for r in batch}})
        # the reference's gap between the k-th and (k+1)-th cosine of each query, for the near-tie check
        qn = emb / np.linalg.norm(emb, axis=1, keepdims=True)
        cn = corpus / np.linalg.norm(corpus, axis=1, keepdims=True)
        s = -np.sort(-(qn.astype(np.float64) @ cn.T.astype(np.float64)), axis=1)
        out_json["batches"][-1]["min_gap"] = float(min(s[i, k - 1] - s[i, k] for i, k in enumerate(ks)
                                                       if 0 < k < s.shape[1]))
        print(f"batch {bi}: B={len(batch)} min gap {out_json['batches'][-1]['min_gap']:.3g}", flush=True)
    tag = "" if corpus_name == "short_facts" else f"_{corpus_name}"
    np.savez_compressed(os.path.join(HERE, f"golden_embed{tag}.npz"), **out_npz)
    with open(os.path.join(HERE, f"golden_embed{tag}.json"), "w") as f:
        json.dump(out_json, f)
    print("reference:", REF, "done")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "short_facts")
