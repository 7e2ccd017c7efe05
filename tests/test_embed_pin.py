"""The embedding half against the reference's own BatchProcessor._process_batch
(tests/golden/golden_embed.*, made by make_embed_golden.py with the stand-in models of embed_fixture.py):
the (B, 1024) array handed to batch_retrieve, the prompts and the stored results.

CPU: our embed_queries reproduces the reference's embeddings, and our _process_batch — fed the
reference's documents — builds the same prompts and stores the same results.
GPU: the full path (encoder on cuda:0, HipRetriever over short_facts and over the SQuAD corpus — BASELINE
config 4's — device hand-off and host round trip) stores exactly the reference's results."""
import json
import os

import numpy as np
import pytest

import embed_fixture as fx

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "golden", "data")


def load_golden(corpus="short_facts"):
    tag = "" if corpus == "short_facts" else f"_{corpus}"
    with open(os.path.join(HERE, "golden", f"golden_embed{tag}.json")) as f:
        g = json.load(f)
    emb = np.load(os.path.join(HERE, "golden", f"golden_embed{tag}.npz"))
    for i, b in enumerate(g["batches"]):
        b["emb"] = emb[f"emb{i}"]
    return g


def load_queries(corpus="short_facts"):
    return json.load(open(os.path.join(DATA, f"{corpus}_queries.json")))


@pytest.fixture(scope="module")
def golden():
    return load_golden()


@pytest.fixture(scope="module")
def queries():
    return load_queries()


class _Queue:
    def __init__(self):
        self.results = {}

    def store_result(self, rid, result):
        self.results[rid] = result


def test_embeddings_match_reference_cpu(golden, queries):
    import torch
    from rag_service_amd.core.batch_processor import embed_queries
    model = {"tokenizer": fx.HashTokenizer(), "model": fx.make_encoder()}
    for batch, g in zip(fx.batches(queries), golden["batches"]):
        got = embed_queries(model, [r["query"] for r in batch], torch.device("cpu")).numpy()
        assert got.shape == g["emb"].shape
        np.testing.assert_allclose(got, g["emb"], rtol=0, atol=1e-6)


def test_prompts_and_results_match_reference_cpu(golden, queries):
    from rag_service_amd.core.batch_processor import BatchProcessor

    class ReplayRetriever:
        """Checks the hand-off and answers with the reference's documents for that batch."""
        devices = [0]

        def __init__(self):
            self.i = 0

        def batch_retrieve(self, q, ks):
            g = golden["batches"][self.i]
            self.i += 1
            np.testing.assert_allclose(q, g["emb"], rtol=0, atol=1e-6)
            assert list(ks) == g["ks"]
            return g["docs"]

    llm = fx.EchoLLM()
    q = _Queue()
    proc = BatchProcessor(q, {"tokenizer": fx.HashTokenizer(), "model": fx.make_encoder()}, llm,
                          ReplayRetriever(), device="cpu")
    for bi, batch in enumerate(fx.batches(queries)):
        proc._process_batch(batch)
        assert llm.prompts[bi] == golden["batches"][bi]["prompts"]
        for rid, res in golden["batches"][bi]["results"].items():
            assert q.results[rid] == res


def test_squad_golden_embeddings_match_cpu():
    """The SQuAD-corpus golden (config 4's corpus; reference _process_batch with the SQuAD questions): our
    embed_queries reproduces its (B, 1024) arrays on CPU."""
    import torch
    from rag_service_amd.core.batch_processor import embed_queries
    golden, queries = load_golden("squad"), load_queries("squad")
    model = {"tokenizer": fx.HashTokenizer(), "model": fx.make_encoder()}
    for batch, g in zip(fx.batches(queries), golden["batches"]):
        got = embed_queries(model, [r["query"] for r in batch], torch.device("cpu")).numpy()
        np.testing.assert_allclose(got, g["emb"], rtol=0, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("corpus_name", ["short_facts", "squad"])
@pytest.mark.parametrize("handoff", [True, False])
def test_process_batch_matches_reference_gpu(hip, handoff, corpus_name):
    """BatchProcessor + HipRetriever store exactly what the reference's _process_batch stored, over the
    short_facts corpus and over BASELINE config 4's SQuAD corpus (batch_processor.py:74-97)."""
    import torch
    from rag_service_amd.core.batch_processor import BatchProcessor, embed_queries
    from rag_service_amd.core.retriever import HipRetriever
    golden, queries = load_golden(corpus_name), load_queries(corpus_name)
    corpus = np.load(os.path.join(DATA, f"{corpus_name}_embeddings.npy"))
    contexts = json.load(open(os.path.join(DATA, f"{corpus_name}_contexts.json")))
    retr = HipRetriever(corpus, contexts)
    model = {"tokenizer": fx.HashTokenizer(), "model": fx.make_encoder()}
    llm = fx.EchoLLM()
    q = _Queue()
    proc = BatchProcessor(q, model, llm, retr, device="cuda:0", device_handoff=handoff)
    for bi, batch in enumerate(fx.batches(queries)):
        g = golden["batches"][bi]
        emb = embed_queries(model, [r["query"] for r in batch], torch.device("cuda:0")).cpu().numpy()
        np.testing.assert_allclose(emb, g["emb"], rtol=0, atol=1e-5)     # GPU vs CPU fp32 encoder
        proc._process_batch(batch)
        assert llm.prompts[bi] == g["prompts"]
        for rid, res in g["results"].items():
            assert q.results[rid] == res, rid
    retr.close()
