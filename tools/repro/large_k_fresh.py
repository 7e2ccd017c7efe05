import sys, numpy as np
sys.path[:0] = [".", "rag-serving-system_amd"]
import torch; torch.cuda.is_available()
from rag_service_amd import Index
from oracle.retriever_oracle import canonical_topk, exact_scores
rng = np.random.default_rng(8)
corpus = rng.standard_normal((20000, 1024)).astype(np.float32)
q = rng.standard_normal((32, 1024)).astype(np.float32)
_, cidx = canonical_topk(exact_scores(corpus, q, "cosine"), 100)
for order in ("exact-first", "wide-first"):
    ix = Index(dtype="fp32", metric="cosine"); ix.load(corpus)
    seq = ["exact", "auto"] if order == "exact-first" else ["auto", "exact"]
    for kern in seq:
        ix.set_kernel(kern)
        s, i = ix.search(q, 100)
        print(order, kern, "match", np.mean(i == cidx), "scores", s[0, :3], i[0, :4], flush=True)
    ix.close()
ix = Index(dtype="fp32", metric="cosine"); ix.load(corpus); ix.set_kernel("exact")
for k in (33, 100):
    s, i = ix.search(q, k)
    print("fresh exact k", k, np.mean(i == cidx[:, :k]), s[0, :3], flush=True)
