"""BatchProcessor drop-in: the embedding half's semantics (batch_processor.py:74-125) on CPU with a
small torch model, and (GPU) the device-pointer hand-off into the HIP retriever."""
import numpy as np
import pytest
import torch

from rag_service_amd.core.batch_processor import BatchProcessor, embed_queries


class _Tok:
    """Whitespace tokenizer with right padding (pad id 0) and truncation to 16 tokens."""
    def __call__(self, texts, padding=True, truncation=True, return_tensors="pt"):
        ids = [[(hash(w) % 997) + 1 for w in t.split()][:16] for t in texts]
        L = max(len(x) for x in ids)
        pad = [x + [0] * (L - len(x)) for x in ids]
        mask = [[1] * len(x) + [0] * (L - len(x)) for x in ids]
        self.last = texts
        return {"input_ids": torch.tensor(pad), "attention_mask": torch.tensor(mask)}


class _Enc(torch.nn.Module):
    def __init__(self, dim=64):
        super().__init__()
        torch.manual_seed(0)
        self.emb = torch.nn.Embedding(1000, dim)

    def forward(self, input_ids, attention_mask):
        class O:  # HF-style output object
            pass
        o = O()
        o.last_hidden_state = self.emb(input_ids)
        return o


class _Queue:
    def __init__(self, batches):
        self.batches, self.results = list(batches), {}

    def get_batch(self):
        return self.batches.pop(0) if self.batches else []

    def store_result(self, rid, res):
        self.results[rid] = res


class _Retr:
    def __init__(self):
        self.calls = []

    def batch_retrieve(self, q, ks):
        self.calls.append((q, ks))
        return [[f"doc{i}-{j}" for j in range(k)] for i, k in enumerate(ks)]


PROMPTS = []


def _llm(prompts, max_new_tokens, do_sample, batch_size):
    assert max_new_tokens == 10 and do_sample and batch_size == len(prompts)
    PROMPTS[:] = prompts
    return [f"answer:{i}" for i in range(len(prompts))]


def test_embedding_semantics_mean_includes_padding():
    tok, enc = _Tok(), _Enc()
    emb = embed_queries({"tokenizer": tok, "model": enc}, ["a b c", "d"], torch.device("cpu"))
    assert tok.last == ["query: a b c", "query: d"]
    ids = tok(["query: a b c", "query: d"])["input_ids"]
    want = enc.emb(ids).mean(dim=1)            # pad positions included, no L2 normalisation
    assert torch.allclose(emb, want)
    assert not torch.allclose(emb.norm(dim=1), torch.ones(2))


def test_process_batch_end_to_end_cpu():
    q = _Queue([[{"id": "r1", "query": "x y", "k": 2}, {"id": "r2", "query": "z", "k": 3}]])
    retr = _Retr()
    bp = BatchProcessor(q, {"tokenizer": _Tok(), "model": _Enc()}, _llm, retr, device="cpu")
    bp._process_batch(q.get_batch())
    (emb, ks), = retr.calls
    assert isinstance(emb, np.ndarray) and emb.shape == (2, 64) and ks == [2, 3]
    assert q.results["r1"]["result"] == "answer:0"
    assert PROMPTS[0] == "Context:\ndoc0-0\n---\ndoc0-1\n\nQuestion: x y\n\nThe Answer to this question is: "
    assert set(q.results) == {"r1", "r2"}


def test_process_batch_error_path():
    q = _Queue([])
    bp = BatchProcessor(q, {"tokenizer": _Tok(), "model": _Enc()}, lambda *a, **k: 1 / 0, _Retr(), device="cpu")
    bp._process_batch([{"id": "r1", "query": "x", "k": 1}])
    assert q.results["r1"]["status"] == "failed" and "division" in q.results["r1"]["error"]


def test_run_loop_processes_then_stops():
    q = _Queue([[{"id": "a", "query": "x", "k": 1}]])
    bp = BatchProcessor(q, {"tokenizer": _Tok(), "model": _Enc()}, _llm, _Retr(), device="cpu",
                        polling_interval=0.01)
    bp.start()
    import time
    for _ in range(200):
        if "a" in q.results:
            break
        time.sleep(0.01)
    bp.stop()
    bp.join(timeout=5)
    assert "a" in q.results and not bp.is_alive()


@pytest.mark.gpu
def test_device_handoff_matches_host_path(hip, squad):
    from rag_service_amd.core.retriever import HipRetriever
    from oracle.retriever_oracle import cupy_batch_retrieve
    docs = [f"doc{i}" for i in range(squad.shape[0])]
    retr = HipRetriever(squad, docs)
    enc = _Enc(dim=1024)
    queue = _Queue([])
    queries = [f"question number {i} about topic {i % 7}" for i in range(32)]
    ks = [5] * 16 + [2] * 16
    dev = BatchProcessor(queue, {"tokenizer": _Tok(), "model": enc}, _llm, retr, device="cuda:0")
    got_dev = dev.retrieve(queries, ks)
    host = BatchProcessor(queue, {"tokenizer": _Tok(), "model": enc}, _llm, retr, device="cuda:0",
                          device_handoff=False)
    got_host = host.retrieve(queries, ks)
    assert got_dev == got_host
    emb = embed_queries({"tokenizer": _Tok(), "model": enc}, queries, torch.device("cuda:0")).cpu().numpy()
    want = cupy_batch_retrieve(squad, emb, ks)
    assert [[int(d[3:]) for d in row] for row in got_dev] == want
