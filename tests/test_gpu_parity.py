"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors and the oracle.

Golden vectors come from the reference retrievers themselves (tests/golden/make_golden.py). Sizes the
oracle handles in seconds are compared directly; the 1M-row cases compare against the reference's
committed outputs, plus size-independent properties (self-retrieval, bf16/fp32 agreement on the
exact-integer corpus, determinism).
"""
import numpy as np
import pytest

from oracle import synth
from oracle.retriever_oracle import canonical_topk, exact_scores
from parity_helpers import check_topk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Index(hip):
    from rag_service_amd import Index as _Index
    return _Index


_cache = {}


def get_index(Index, key, corpus, dtype="fp32", metric="cosine"):
    k = (key, dtype, metric)
    if k not in _cache:
        ix = Index(dtype=dtype, metric=metric)
        ix.load(corpus)
        _cache[k] = ix
    return _cache[k]


GOLDEN_CASES = [
    ("sf_self_k1", "sf", "sf_self", 1), ("sf_self_k5", "sf", "sf_self", 5), ("sf_self_k10", "sf", "sf_self", 10),
    ("sf_rand_k1", "sf", "rand", 1), ("sf_rand_k5", "sf", "rand", 5), ("sf_rand_k10", "sf", "rand", 10),
    ("sf_rand_k100", "sf", "rand", 100),
    ("sq_rand_k2", "sq", "rand", 2), ("sq_rand_k5", "sq", "rand", 5), ("sq_rand_k10", "sq", "rand", 10),
    ("sq_rand_k32", "sq", "rand", 32), ("sq_rand_k40", "sq", "rand", 40),
    ("sq_self_k5", "sq", "sq_self", 5), ("sq_scaled_k10", "sq", "scaled", 10),
]


def _case_inputs(corpus_key, q_key, short_facts, squad, golden_data):
    corpus = short_facts if corpus_key == "sf" else squad
    queries = {"sf_self": short_facts, "sq_self": squad[:64], "rand": golden_data["rand_queries"],
               "scaled": golden_data["scaled_queries"]}[q_key]
    return corpus, queries


@pytest.mark.parametrize("name,corpus_key,q_key,k", GOLDEN_CASES)
@pytest.mark.parametrize("flavour", ["simple", "cupy"])
def test_golden_reference_data(Index, golden_data, short_facts, squad, name, corpus_key, q_key, k, flavour):
    corpus, queries = _case_inputs(corpus_key, q_key, short_facts, squad, golden_data)
    metric = "dot" if flavour == "simple" else "cosine"
    ix = get_index(Index, corpus_key, corpus, "fp32", metric)
    ref_idx = golden_data[f"{name}_{flavour}_idx"]
    kk = ref_idx.shape[1]
    scores, idx = ix.search(queries, kk)
    exact_rows, near = check_topk(idx, scores, ref_idx, corpus, queries, metric)
    assert exact_rows + near == queries.shape[0]
    if float(golden_data[f"{name}_{flavour}_gap"]) > 1e-5:
        assert near == 0


def test_retriever_classes_match_reference(hip, golden_data, squad):
    from rag_service_amd.core.retriever import HipRetriever, HipSimpleRetriever
    docs = list(range(squad.shape[0]))
    q = golden_data["rand_queries"]
    cupy = HipRetriever(doc_embeddings=squad, documents=docs)
    simple = HipSimpleRetriever(doc_embeddings=squad, documents=docs)
    got_c = cupy.batch_retrieve(q, [10] * q.shape[0])
    got_s = simple.batch_retrieve(q, [10] * q.shape[0])
    assert got_c == golden_data["sq_rand_k10_cupy_idx"].tolist()
    assert got_s == golden_data["sq_rand_k10_simple_idx"].tolist()
    assert cupy.retrieve(q[3], 10) == golden_data["sq_rand_k10_cupy_idx"][3].tolist()
    assert simple.retrieve(q[3:4], 10) == golden_data["sq_rand_k10_simple_idx"][3].tolist()


def test_edge_cases_match_reference(hip, golden_edges, short_facts):
    from rag_service_amd.core.retriever import HipRetriever, HipSimpleRetriever
    n, d = short_facts.shape
    docs = list(range(n))
    rets = {"cupy": HipRetriever(short_facts, docs), "simple": HipSimpleRetriever(short_facts, docs)}
    rng = np.random.default_rng(golden_edges["seed"])
    q4 = rng.standard_normal((4, d)).astype(np.float32)
    q4 /= np.linalg.norm(q4, axis=1, keepdims=True)
    c = golden_edges["cases"]
    batch_inputs = {
        "mixed_ks": (q4, [3, 0, -1, 7]), "k_gt_n": (q4, [n + 50, 2, n, 1]), "all_nonpositive": (q4, [0, -3, 0, -1]),
        "float64_queries": (q4.astype(np.float64), [5] * 4), "wrong_dim": (q4[:, :d - 8], [5] * 4),
        "np_int64_ks": (q4, [np.int64(5)] * 4), "len_mismatch": (q4, [5, 5, 5]), "empty_batch": (q4[:0], []),
        "one_d_batch": (q4[0], [5]),
    }
    for case, (q, ks) in batch_inputs.items():
        for flav, r in rets.items():
            assert r.batch_retrieve(q, ks) == c[case][flav], (case, flav)
    single_inputs = {
        "retrieve_1d": (q4[0], 3), "retrieve_1xd": (q4[:1], 3), "retrieve_k0": (q4[0], 0),
        "retrieve_kneg": (q4[0], -2), "retrieve_k_gt_n": (q4[0], n + 3), "retrieve_2xd": (q4[:2], 3),
        "retrieve_wrong_dim": (q4[0, :d - 8], 3), "retrieve_np_int64_k": (q4[0], np.int64(3)),
        "retrieve_float_k": (q4[0], 2.5), "retrieve_float64": (q4[0].astype(np.float64), 4),
    }
    for case, (q, k) in single_inputs.items():
        for flav, r in rets.items():
            assert r.retrieve(q, k) == c[case][flav], (case, flav)
    with pytest.raises(AttributeError):
        rets["cupy"].batch_retrieve(q4.tolist(), [5] * 4)
    assert c["cupy_list_input"] == "AttributeError"


# ---- synthetic corpora (64k rows: reference outputs committed; oracle-checkable) ----------------------
@pytest.fixture(scope="module")
def f2_small(golden_synth):
    seed, qseed, _, n = [int(x) for x in golden_synth["meta"]]
    return synth.exact_int_rows(seed, 0, n, 1024), synth.exact_int_queries(qseed, 32, 1024)


@pytest.fixture(scope="module")
def f3_small(golden_synth):
    seed, _, qseed, n = [int(x) for x in golden_synth["meta"]]
    return synth.unit_norm_gaussian(seed, n, 1024), synth.unit_norm_gaussian(qseed, 32, 1024)


def test_fp32_split_storage_round_trip(Index):
    """RR_DTYPE_F32_SPLIT keeps x as f16 hi + lo with a per-row power-of-two scale: read-back is within 2^-22
    relative of every input element (22-bit significand), exact for values with <= 22 significant bits."""
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((257, 128)) * rng.uniform(1e-3, 1e3, size=(257, 1))).astype(np.float32)
    x[3] = 0.0
    ix = Index(dtype="fp32-split", metric="dot")
    ix.load(x)
    y = ix.read_rows(0, 257)
    bound = 2.0 ** -22 * np.abs(x) + 2.0 ** -30 * np.abs(x).max(axis=1, keepdims=True)   # tiny elements: f16 subnormal lo
    assert np.all(np.abs(y - x) <= bound)
    ints = synth.exact_int_rows(3, 0, 64, 128)
    ix.load(ints)
    assert np.array_equal(ix.read_rows(0, 64), ints)


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_pipelined_ingest_multi_chunk(Index, dtype):
    """rr_load streams the host array through two pinned 32 MiB staging buffers (8192 rows of d = 1024 per
    chunk): 3 full chunks + a ragged one must land exactly (exact-integer rows are exact in every storage
    dtype) and search identically to the same rows generated on the device."""
    n = 3 * 8192 + 17
    rows = synth.exact_int_rows(99, 0, n, 1024)
    ix = Index(dtype=dtype, metric="cosine")
    ix.load(rows)
    for r0 in (0, 8190, 16384, n - 20):
        assert np.array_equal(ix.read_rows(r0, 20), rows[r0:r0 + 20])
    gen = Index(dtype=dtype, metric="cosine")
    gen.fill_synthetic(0, 99, n, 1024)
    q = rows[[5, 8192, 16385, n - 1]]
    s1, i1 = ix.search(q, 5)
    s2, i2 = gen.search(q, 5)
    assert np.array_equal(i1, i2) and np.array_equal(s1, s2)
    assert list(i1[:, 0]) == [5, 8192, 16385, n - 1]
    sh = Index(devices=[0, 0], dtype=dtype, metric="cosine")   # two shards, each its own pipelined upload
    sh.load(rows)
    s3, i3 = sh.search(q, 5)
    assert np.array_equal(i1, i3) and np.array_equal(s1, s3)


def test_device_generator_matches_numpy(Index, golden_synth):
    ix = Index(dtype="fp32", metric="dot")
    ix.fill_synthetic(0, 1234, 4099, 1024)
    assert np.array_equal(ix.read_rows(0, 4099), synth.exact_int_rows(1234, 0, 4099, 1024))
    ix2 = Index(dtype="fp32", metric="dot")
    ix2.fill_synthetic(1, 77, 300, 1024)
    ref = synth.irwin_hall_unnormalised(77, 0, 300, 1024)
    ref /= np.linalg.norm(ref, axis=1, keepdims=True)
    np.testing.assert_allclose(ix2.read_rows(0, 300), ref, rtol=0, atol=2e-7)


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_exact_integer_corpus_bit_exact(Index, golden_synth, f2_small, dtype):
    """F2: every dot is exact in fp32, so scores must equal the fp64 values bit-for-bit and the order is
    the canonical (score desc, index asc); where the reference had no ties its order matches too."""
    corpus, q = f2_small
    ix = get_index(Index, "f2_small", corpus, dtype, "dot")
    scores, idx = ix.search(q, 10)
    val, cidx = canonical_topk(exact_scores(corpus, q, "dot"), 10)
    assert np.array_equal(scores.astype(np.float64), val)
    assert np.array_equal(idx, cidx)
    ref = golden_synth["f2_64k_k10_simple_idx"]
    ex = exact_scores(corpus, q, "dot")
    for i in range(q.shape[0]):
        s = np.sort(ex[i])[::-1][:11]
        if np.all(np.diff(s) != 0):
            assert np.array_equal(idx[i], ref[i])


@pytest.mark.parametrize("metric,flav", [("dot", "simple"), ("cosine", "cupy")])
@pytest.mark.parametrize("dtype", ["fp32", "fp32-split"])
def test_unit_norm_corpus_fp32(Index, golden_synth, f3_small, metric, flav, dtype):
    corpus, q = f3_small
    ix = get_index(Index, "f3_small", corpus, dtype, metric)
    scores, idx = ix.search(q, 10)
    check_topk(idx, scores, golden_synth[f"f3_64k_k10_{flav}_idx"], corpus, q, metric)


@pytest.mark.parametrize("metric,flav", [("dot", "simple"), ("cosine", "cupy")])
def test_unit_norm_corpus_bf16(Index, golden_synth, f3_small, metric, flav):
    corpus, q = f3_small
    ix = get_index(Index, "f3_small", corpus, "bf16", metric)
    rounded = synth.bf16_round(corpus)
    assert np.array_equal(ix.read_rows(0, 64), rounded[:64])
    scores, idx = ix.search(q, 10)
    check_topk(idx, scores, golden_synth[f"f3bf_64k_k10_{flav}_idx"], rounded, q, metric)


# ---- kernel edge cases against the oracle's canonical top-k -----------------------------------------
SHAPES = [  # (n, d, b, k)
    (1, 64, 1, 1), (31, 64, 3, 5), (33, 128, 32, 4), (100, 1024, 33, 8), (1000, 1024, 70, 17),
    (4097, 256, 5, 32), (5000, 128, 2, 33), (777, 64, 9, 64), (50, 128, 4, 80), (20000, 1024, 32, 16),
    (3001, 512, 17, 10), (2500, 768, 32, 3), (40000, 1024, 8, 32),
]


@pytest.mark.parametrize("n,d,b,k", SHAPES)
@pytest.mark.parametrize("metric", ["dot", "cosine"])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_shapes_against_oracle(Index, n, d, b, k, metric, dtype):
    if dtype == "bf16" and d % 128:
        pytest.skip("bf16 path needs d % 128 == 0")
    rng = np.random.default_rng(n * 31 + d + b + k)
    corpus = rng.standard_normal((n, d)).astype(np.float32) * rng.uniform(0.5, 2, size=(n, 1)).astype(np.float32)
    q = rng.standard_normal((b, d)).astype(np.float32)
    if dtype == "bf16":
        corpus = synth.bf16_round(corpus)
    ix = Index(dtype=dtype, metric=metric)
    ix.load(corpus)
    scores, idx = ix.search(q, k)
    _, cidx = canonical_topk(exact_scores(corpus, q, metric), k)
    tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
    check_topk(idx, scores, cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
    if k > n:
        assert np.all(idx[:, n:] == -1) and np.all(np.isneginf(scores[:, n:]))


def test_staged_api_and_determinism(Index, squad, golden_data):
    ix = get_index(Index, "sq", squad, "fp32", "cosine")
    q = golden_data["rand_queries"]
    ix.set_queries(q)
    ix.search_staged(10)
    s1, i1 = ix.fetch()
    for _ in range(3):
        ix.search_staged(10)
    s2, i2 = ix.fetch()
    assert np.array_equal(i1, i2) and np.array_equal(s1, s2)
    s3, i3 = ix.search(q, 10)
    assert np.array_equal(i1, i3)


def test_reused_handle_batch_and_k_changes(Index):
    """One handle, successive synchronous searches whose batch and k grow and shrink (pinned query staging
    and the single-allocation result buffer are re-sized and re-used; k > 32 takes the sort path): every
    result equals a fresh handle's."""
    rng = np.random.default_rng(11)
    corpus = rng.standard_normal((6000, 256)).astype(np.float32)
    ix = Index(dtype="fp32", metric="cosine")
    ix.load(corpus)
    for b, k in [(5, 5), (70, 8), (32, 40), (1, 3), (64, 100), (3, 1), (70, 8)]:
        q = rng.standard_normal((b, 256)).astype(np.float32)
        s1, i1 = ix.search(q, k)
        fresh = Index(dtype="fp32", metric="cosine")
        fresh.load(corpus)
        s2, i2 = fresh.search(q, k)
        fresh.close()
        assert s1.shape == (b, k) and np.array_equal(i1, i2) and np.array_equal(s1, s2)
        _, cidx = canonical_topk(exact_scores(corpus, q, "cosine"), k)
        check_topk(i1, s1, cidx, corpus, q, "cosine", near_tie=1e-5 * 16, score_tol=1e-3)


def test_device_pointer_queries(Index, squad, golden_data):
    torch = pytest.importorskip("torch")
    ix = get_index(Index, "sq", squad, "fp32", "cosine")
    q = golden_data["rand_queries"]
    t = torch.from_numpy(q).to("cuda:0")
    torch.cuda.synchronize()
    ix.set_queries_device(t.data_ptr(), q.shape[0], q.shape[1])
    ix.search_staged(5)
    s, i = ix.fetch()
    s2, i2 = ix.search(q, 5)
    assert np.array_equal(i, i2)


def test_kernel_timing(Index, squad, golden_data):
    ix = get_index(Index, "sq", squad, "fp32", "cosine")
    ix.set_timing(True)
    ix.kernel_time(reset=True)
    ix.search(golden_data["rand_queries"], 5)
    ms, n = ix.kernel_time(reset=True)
    ix.set_timing(False)
    assert n == 1 and ms > 0


def test_errors_are_reported(Index, hip):
    from rag_service_amd import HipRetrievalError
    ix = Index(dtype="fp32", metric="dot")
    with pytest.raises(HipRetrievalError):
        ix.search(np.zeros((1, 64), np.float32), 1)       # no corpus yet
    with pytest.raises(HipRetrievalError):
        ix.load(np.zeros((10, 65), np.float32))            # d not a multiple of 64
    ix.load(np.ones((10, 64), np.float32))
    with pytest.raises(HipRetrievalError):
        ix.search(np.zeros((1, 128), np.float32), 1)      # wrong d
    with pytest.raises(HipRetrievalError):
        ix.search(np.zeros((1, 64), np.float32), 0)       # k < 1


# ---- full size (1M rows) --------------------------------------------------------------------------
@pytest.mark.big
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_1m_exact_integer_against_reference(Index, golden_synth, dtype):
    if "f2_1m_k10_simple_idx" not in golden_synth:
        pytest.skip("1M goldens not generated")
    q = synth.exact_int_queries(99, 32, 1024)
    ix = Index(dtype=dtype, metric="dot")
    ix.fill_synthetic(0, 1234, 1_000_000, 1024)            # bit-identical to synth.exact_int_rows
    for k in (5, 10):
        scores, idx = ix.search(q, k)
        ref = golden_synth[f"f2_1m_k{k}_simple_idx"]
        ref_s = golden_synth[f"f2_1m_k{k}_simple_score"]
        # exact integer arithmetic: scores are bit-exact; indices equal the reference wherever it is
        # tie-free, and otherwise equal the canonical order of the reference's (exact) scores
        assert np.array_equal(np.sort(scores, axis=1), np.sort(ref_s.astype(np.float32), axis=1))
        assert np.array_equal(scores.astype(np.float64), ref_s)
        same = np.all(idx == ref, axis=1)
        for i in np.where(~same)[0]:
            assert len(set(ref_s[i])) < k, f"query {i} differs without ties"


@pytest.mark.big
def test_1m_unit_norm_against_reference(Index, golden_synth):
    if "f3_1m_k10_simple_idx" not in golden_synth:
        pytest.skip("1M goldens not generated")
    corpus = synth.unit_norm_gaussian(1234, 1_000_000, 1024)
    q = synth.unit_norm_gaussian(5678, 32, 1024)
    for metric, flav in (("dot", "simple"), ("cosine", "cupy")):
        ix = Index(dtype="fp32", metric=metric)
        ix.load(corpus)
        for k in (5, 10):
            scores, idx = ix.search(q, k)
            _, near = check_topk(idx, scores, golden_synth[f"f3_1m_k{k}_{flav}_idx"], corpus, q, metric)
            gap = float(golden_synth[f"f3_1m_k{k}_{flav}_gap"])
            print(f"1M unit-norm {metric} k={k}: {near} near-tie rows (recorded gap {gap:.3g})")
            if gap > 1e-5:
                assert near == 0
        # property: self-retrieval — every corpus row finds itself first
        rows = np.arange(0, 1_000_000, 31250)[:32]
        _, sidx = ix.search(corpus[rows], 1)
        assert np.array_equal(sidx[:, 0], rows)
        ix.close()
    bf = synth.bf16_round(corpus)
    del corpus
    ix = Index(dtype="bf16", metric="dot")
    ix.load(bf)
    scores, idx = ix.search(q, 10)
    check_topk(idx, scores, golden_synth["f3bf_1m_k10_simple_idx"], bf, q, "dot")


# ---- row sharding inside one process (several shards on cuda:0, peer-copy exchange) ----------------
@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_sharded_equals_single(Index, shards, dtype):
    """Row shards (rr_create with repeated devices) exchange candidates by peer copy and merge on every
    shard: results must be bit-identical to one shard's for every k path (fused <= 32, sort > 32)."""
    rng = np.random.default_rng(shards * 7 + len(dtype))
    n, d = 5003, 256
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((45, d)).astype(np.float32)     # two 32-query blocks
    for metric in ("dot", "cosine"):
        one = Index(devices=[0], dtype=dtype, metric=metric)
        one.load(corpus)
        many = Index(devices=[0] * shards, dtype=dtype, metric=metric)
        many.load(corpus)
        bounds = [many.shard_range(i) for i in range(shards)]
        per = -(-n // shards)
        assert bounds == [(min(n, i * per), min(n, (i + 1) * per)) for i in range(shards)]
        for k in (1, 5, 32, 40):
            s1, i1 = one.search(q, k)
            s2, i2 = many.search(q, k)
            assert np.array_equal(i1, i2), (metric, k)
            assert np.array_equal(s1, s2), (metric, k)
        one.close()
        many.close()


def test_sharded_more_shards_than_rows(Index):
    corpus = np.arange(3 * 64, dtype=np.float32).reshape(3, 64) / 100.0
    q = np.ones((2, 64), np.float32)
    ix = Index(devices=[0] * 5, dtype="fp32", metric="dot")
    ix.load(corpus)
    for k in (2, 4, 40):
        scores, idx = ix.search(q, k)
        assert list(idx[0][:3]) == [2, 1, 0][:k]
        assert np.all(idx[:, 3:] == -1)


def test_sharded_staged_repeat_and_synthetic(Index):
    """Back-to-back staged searches reuse the exchange buffers (event ordering), and the device
    generator fills each shard from global row indices."""
    one = Index(devices=[0], dtype="fp32", metric="cosine")
    one.fill_synthetic(1, 42, 20000, 512)
    many = Index(devices=[0, 0, 0, 0], dtype="fp32", metric="cosine")
    many.fill_synthetic(1, 42, 20000, 512)
    q = np.random.default_rng(1).standard_normal((32, 512)).astype(np.float32)
    ref = one.search(q, 8)
    many.set_queries(q)
    for _ in range(20):
        many.search_staged(8)
    s, i = many.fetch()
    assert np.array_equal(i, ref[1]) and np.array_equal(s, ref[0])
    assert np.array_equal(many.read_rows(9999, 3), one.read_rows(9999, 3))


# ---- the two similarity kernels (split-K LDS-DMA vs register streaming) ------------------------------
SK_SHAPES = [  # (n, d, b, k): split-K eligible for fp32 / fp32-split at d % 256 == 0, bf16 at d % 512 == 0
    (1, 256, 1, 1), (33, 256, 3, 4), (1000, 512, 32, 8), (31, 1024, 32, 5), (12345, 1024, 20, 16),
    (2049, 768, 7, 32), (70000, 1024, 32, 5),
]


@pytest.mark.parametrize("n,d,b,k", SK_SHAPES)
@pytest.mark.parametrize("metric", ["dot", "cosine"])
@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_split_k_kernel_matches_register_kernel_and_oracle(Index, n, d, b, k, metric, dtype):
    if dtype == "bf16" and d % 512:
        pytest.skip("split-K bf16 needs d % 512 == 0")
    rng = np.random.default_rng(n + 7 * d + b + k)
    corpus = rng.standard_normal((n, d)).astype(np.float32) * rng.uniform(0.5, 2, size=(n, 1)).astype(np.float32)
    q = rng.standard_normal((b, d)).astype(np.float32)
    if dtype == "bf16":
        corpus = synth.bf16_round(corpus)
    ix = Index(dtype=dtype, metric=metric)
    ix.load(corpus)
    s_sk, i_sk = ix.search(q, k)
    ix.set_kernel("fused")
    s_rk, i_rk = ix.search(q, k)
    _, cidx = canonical_topk(exact_scores(corpus, q, metric), k)
    tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
    for idx, scores in ((i_sk, s_sk), (i_rk, s_rk)):
        check_topk(idx, scores, cidx, corpus, q, metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
    agree = np.mean(i_sk == i_rk)
    assert agree >= 0.98, agree
    np.testing.assert_allclose(s_sk, s_rk, rtol=0, atol=2e-5 * (np.sqrt(d) if metric == "dot" else 1.0))


@pytest.mark.parametrize("dtype", ["fp32", "bf16", "fp32-split"])
def test_split_k_exact_integer_bit_exact(Index, golden_synth, f2_small, dtype):
    """Exact-integer corpus: the split-K kernel's K-partial sums are exact, so scores equal fp64."""
    corpus, q = f2_small
    ix = get_index(Index, "f2_small", corpus, dtype, "dot")
    for kernel in ("auto", "fused"):
        ix.set_kernel(kernel)
        scores, idx = ix.search(q, 10)
        val, cidx = canonical_topk(exact_scores(corpus, q, "dot"), 10)
        assert np.array_equal(scores.astype(np.float64), val), kernel
        assert np.array_equal(idx, cidx), kernel
    ix.set_kernel("auto")


def test_split_k_fp32_error_is_fp32_class(Index):
    """fp32 storage through the split-K kernel (exact three-way bf16 split, 6 MFMAs): score error against
    fp64 stays within a few fp32 roundings of sum |x q| — the same class as an fp32 FMA chain."""
    rng = np.random.default_rng(11)
    n, d = 4096, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((32, d)).astype(np.float32)
    ix = Index(dtype="fp32", metric="dot")
    ix.load(corpus)
    scores, idx = ix.search(q, 32)
    ix.set_kernel("fused")
    s_f, i_f = ix.search(q, 32)
    c64, q64 = corpus.astype(np.float64), q.astype(np.float64)
    for sc, ii in ((scores, idx), (s_f, i_f)):
        exact = np.einsum("bd,bkd->bk", q64, c64[ii])
        mag = np.einsum("bd,bkd->bk", np.abs(q64), np.abs(c64[ii]))
        rel = np.abs(sc - exact) / mag
        assert rel.max() < 2.0 ** -19, rel.max()


def test_sharded_pipelined_exchange_mixed_k(Index):
    """Back-to-back staged searches alternate the pipelined exchange (k <= 32: second stream, parity
    buffers) with the serial k > 32 path; every fetch must equal the single-shard result."""
    rng = np.random.default_rng(21)
    corpus = rng.standard_normal((9001, 256)).astype(np.float32)
    q = rng.standard_normal((40, 256)).astype(np.float32)
    one = Index(devices=[0], dtype="fp32", metric="cosine")
    one.load(corpus)
    many = Index(devices=[0, 0, 0], dtype="fp32", metric="cosine")
    many.load(corpus)
    many.set_queries(q)
    for k in (5, 40, 8, 8, 33, 1, 32, 32, 32, 2):
        want = one.search(q, k)
        for _ in range(3):
            many.search_staged(k)
        s, i = many.fetch()
        assert np.array_equal(i, want[1]) and np.array_equal(s, want[0]), k
    one.close()
    many.close()


# ---- 64 query slots per corpus pass (bf16 / fp32-split storage, k <= 16) ------------------------------
@pytest.mark.parametrize("dtype", ["bf16", "fp32-split"])
@pytest.mark.parametrize("metric", ["dot", "cosine"])
def test_split_k_64_query_slots(Index, dtype, metric):
    """b in 33..64 runs ONE split-K pass with 64 query slots (BASELINE config 5 is batch 64): results are
    bit-identical to 32-query passes over the same queries and match the oracle's canonical top-k."""
    rng = np.random.default_rng(64 + len(dtype))
    n, d = 12345, 1024
    corpus = rng.standard_normal((n, d)).astype(np.float32)
    if dtype == "bf16":
        corpus = synth.bf16_round(corpus)
    q = rng.standard_normal((100, d)).astype(np.float32)
    ix = Index(dtype=dtype, metric=metric)
    ix.load(corpus)
    ex = exact_scores(corpus, q, metric)
    tol = 1e-3 * (np.sqrt(d) if metric == "dot" else 1.0)
    for b in (33, 64, 100):
        for k in (1, 5, 16, 17):
            ix.set_timing(True)
            ix.kernel_time(reset=True)
            s64, i64 = ix.search(q[:b], k)
            _, launches = ix.kernel_time(reset=True)
            ix.set_timing(False)
            if k <= 16:
                assert launches == -(-b // 64), (b, k, launches)
            parts = [ix.search(q[q0:min(b, q0 + 32)], k) for q0 in range(0, b, 32)]
            assert np.array_equal(i64, np.concatenate([p[1] for p in parts])), (b, k)
            assert np.array_equal(s64, np.concatenate([p[0] for p in parts])), (b, k)
            _, cidx = canonical_topk(ex[:b], k)
            check_topk(i64, s64, cidx, corpus, q[:b], metric, near_tie=1e-5 * np.sqrt(d), score_tol=tol)
    ix.close()


def test_split_k_64_slots_sharded(Index):
    """64-slot passes through the pipelined cross-shard exchange equal the single-shard result."""
    rng = np.random.default_rng(7)
    corpus = synth.bf16_round(rng.standard_normal((20011, 1024)).astype(np.float32))
    q = rng.standard_normal((64, 1024)).astype(np.float32)
    one = Index(devices=[0], dtype="bf16", metric="cosine")
    one.load(corpus)
    many = Index(devices=[0, 0, 0, 0], dtype="bf16", metric="cosine")
    many.load(corpus)
    for k in (5, 10, 40):
        a, b = one.search(q, k), many.search(q, k)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0]), k
    one.close()
    many.close()
