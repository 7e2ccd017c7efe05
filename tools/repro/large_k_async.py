import sys, numpy as np
sys.path[:0] = [".", "rag-serving-system_amd"]
import torch; torch.cuda.is_available()
from rag_service_amd import Index
from oracle.retriever_oracle import canonical_topk, exact_scores
rng = np.random.default_rng(8)
corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
ix = Index(dtype="fp32", metric="cosine"); ix.load(corpus)
ref = Index(dtype="fp32", metric="cosine"); ref.load(corpus); ref.set_kernel("exact")
qs = [rng.standard_normal((32, 1024)).astype(np.float32) for _ in range(4)]
c = [canonical_topk(exact_scores(corpus, q, "cosine"), 100)[1] for q in qs]
mode = sys.argv[1]
if mode == "ref-first":
    s, i = ref.search(qs[0], 100); print("ref first", np.mean(i == c[0]), s[0, :3], flush=True)
tickets = [ix.search_async(q, 100) for q in qs]
for j, t in enumerate(tickets):
    s, i = ix.wait(t); print("ix", j, np.mean(i == c[j]), s[0, :2], flush=True)
    s, i = ref.search(qs[j], 100); print("ref", j, np.mean(i == c[j]), s[0, :2], flush=True)
