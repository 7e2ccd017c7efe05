"""CPU restatement of the int8 screens' bound (rr_kernels.hip f32_to_i8_kernel / q8_prep_kernel / q9_prep_kernel,
rr_sk.hip DT 8 and DT 9 epilogues — DT 9: bf16 storage's screen, the rows' bf16 roundings against ONE query piece) in
float32 numpy, checked against float64 dot products: the bound must hold for every row, including rows
the int8 copy represents badly (a spike sets the scale and every other element rounds to zero), zero rows, tiny and
huge magnitudes. This pins the ALGEBRA of the bound (Cauchy-Schwarz on the two residuals); the GPU tests
(test_gpu_int8.py) pin the kernels against the exact kernel."""
import numpy as np
import pytest

F = np.float32


def quantize_rows(x):
    """f32_to_i8_kernel: t = x / sx, x8 = clamp(rint(t)); e from the scaled residual t - x8 (exact), so no square
    underflows: e = sx |t - x8| (1 + 2^-12) + 2^-22 sqrt(d) max|x| + 2^-140."""
    m = np.abs(x).max(axis=1)
    s = np.where(m > 0, m / F(127), F(0)).astype(F)
    with np.errstate(divide="ignore", invalid="ignore", under="ignore"):
        t = np.where(s[:, None] > 0, x / s[:, None], F(0)).astype(F)
        q = np.clip(np.rint(t), -127, 127).astype(F)
        r = (t - q).astype(F)
        e = ((s * np.sqrt((r * r).sum(axis=1, dtype=F))).astype(F) * F(1 + 2 ** -12)
             + (m * F(np.sqrt(x.shape[1]) * 2 ** -22) + F(2 ** -140))).astype(F)
    return q.astype(np.int8), s, e


def quantize_query(v, pieces=2):
    """The staged pieces (rr_device.h q8_stage_row, once per staged batch): t = q / s, p1 = clamp(rint(t)),
    p2 = clamp(rint((t - p1) 64)); eq from the exact scaled residual t - p1 - p2 / 64. pieces = 1 (DT 9 reads p1 and
    the one-piece scalars of the same staging): p2 = 0, the residual t - p1, the scale s itself."""
    m = F(np.abs(v).max())
    s = F(m / F(127)) if m > 0 else F(0)
    with np.errstate(under="ignore"):
        if s > 0:
            t = (v / s).astype(F)
            a = np.clip(np.rint(t), -127, 127).astype(F)
            ta = (t - a).astype(F)
            if pieces == 2:
                c = np.clip(np.rint(ta * F(64)), -127, 127).astype(F)
                r = (ta - c * F(2 ** -6)).astype(F)
            else:
                c = np.zeros_like(v)
                r = ta
        else:
            a = c = r = np.zeros_like(v)
        eq = F(F(s * np.sqrt((r * r).sum(dtype=F))) * F(1 + 2 ** -12)
               + (m * F(np.sqrt(v.size) * 2 ** -21) + F(2 ** -140)))
        qn = F(np.sqrt((v * v).sum(dtype=F)))
        qsa = F(np.abs(v).sum(dtype=F) * F(1 + 2 ** -18))
        if pieces == 1:   # (the DT 9 MFMA sums x8 . p1: the bound's "64 p1 + p2" with p1 taken once and p2 = 0)
            return a.astype(np.int8), c.astype(np.int8), F(s), eq, qn, qsa, 1
        return a.astype(np.int8), c.astype(np.int8), F(s * F(2 ** -6)), eq, qn, qsa, 64


def bound(xq, sx, e, nd, p1, p2, qsc, eq, qn, qsa, w1=64, eps_a=6e-5, eps_b=4e-8):
    """The DT 8 / DT 9 epilogue's upper bound of x . q (nd: the fp32 row norm the kernel reads, short when squares
    underflow; w1: the first piece's weight, 64 with two pieces, 1 with one)."""
    acc = xq.astype(np.int64) @ (w1 * p1.astype(np.int64) + p2.astype(np.int64))   # exact, as the int32 MFMA sums
    s = acc.astype(F)
    est = (s * sx).astype(F) * qsc
    sqrt_d = F(np.sqrt(xq.shape[1]) * (1 + 2 ** -20))
    # the kernel's factored form: e Q1 + |x| Q2 + Q3 with per-query Q1 = (|q| + eq), Q2 = eq + eps_a |q| + eps_b sqrt(d),
    # Q3 = eps_b sum|q|, each x 1.001
    q1 = F((qn + eq) * F(1.001))
    q2 = F((eq + (F(eps_a) * qn + F(eps_b) * sqrt_d)) * F(1.001))
    # (+ the absolute 2^-110 and Q2 2^-69 for row norms whose squares underflow, rr_sk.hip q8e3)
    q3 = F(q2 * F(2 ** -69) + (F(eps_b) * qsa * F(1.001) + F(2 ** -110)))
    eps = (e * q1 + (nd * q2 + q3)).astype(F)
    v = est + np.abs(est) * F(2 ** -21) + eps
    return v + np.abs(v) * F(2 ** -22)


KINDS = ["gauss", "spiky", "scaled", "tiny", "small", "huge", "zero_rows", "sparse",
         # rows AND queries tiny together: the scales' product sx q8sc, the estimate and the
         # residual terms fall into fp32's subnormal range
         "both_2^-60", "both_2^-64", "rows_2^-100_q_2^-30", "rows_2^-30_q_2^-100", "rows_2^-120"]


def bf16_round(x):
    """fp32 -> its bf16 rounding (RNE), as fp32: the values bf16 storage holds (f32_to_i8_kernel's bf16 = 1 quantises
    them, and the verify's exact score is of them)."""
    u = np.ascontiguousarray(x, dtype=F).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(F)


@pytest.mark.parametrize("pieces", [2, 1])
@pytest.mark.parametrize("kind", KINDS)
def test_int8_bound_holds(kind, pieces):
    """pieces 2: DT 8 (fp32 rows); pieces 1: DT 9 (the rows' bf16 roundings; their exact score is of those values)."""
    rng = np.random.default_rng(sum(map(ord, kind)))
    n, d = 3000, 1024
    x = rng.standard_normal((n, d)).astype(F)
    qscale = 1.0
    if kind == "spiky":
        x *= F(0.05)
        x[np.arange(n), rng.integers(0, d, n)] = F(60.0)
    elif kind == "scaled":
        x *= rng.uniform(1e-3, 1e3, size=(n, 1)).astype(F)
    elif kind == "tiny":
        x *= F(1e-30)
    elif kind == "small":   # squared residuals below fp32's range (e reads 0), queries of normal size
        x *= F(1e-20)
    elif kind == "huge":
        x *= F(1e4)
    elif kind == "zero_rows":
        x[::3] = 0
    elif kind == "sparse":
        x[rng.random((n, d)) < 0.97] = 0
    elif kind.startswith("both_"):
        e = int(kind.split("^")[1])
        x = (x.astype(np.float64) * 2.0 ** e).astype(F)
        qscale = 2.0 ** e
    elif kind.startswith("rows_"):
        parts = kind.split("_")
        x = (x.astype(np.float64) * 2.0 ** int(parts[1].split("^")[1])).astype(F)
        if len(parts) > 2:
            qscale = 2.0 ** int(parts[3].split("^")[1])
    if pieces == 1:
        with np.errstate(over="ignore"):
            x = bf16_round(x)
    xq, sx, e = quantize_rows(x)
    with np.errstate(under="ignore"):   # the fp32 norm the kernels read (row_norms_kernel): squares may underflow
        nd = np.sqrt((x * x).sum(axis=1, dtype=F)).astype(F)
    for j in range(8):
        v = rng.standard_normal(d).astype(F)
        if j % 2:   # queries aligned with some rows (their true matches)
            v = (x[rng.integers(n)] + F(0.1) * np.abs(x).max() * rng.standard_normal(d).astype(F)).astype(F)
            v = (v.astype(np.float64) / max(float(np.abs(v).max()), 1e-300)).astype(F)
        v = (v.astype(np.float64) * qscale).astype(F)
        with np.errstate(under="ignore"):
            u = bound(xq, sx, e, nd, *quantize_query(v, pieces))
        exact = x.astype(np.float64) @ v.astype(np.float64)
        assert np.all(u.astype(np.float64) >= exact), float(np.max(exact - u))


def test_int8_bound_is_about_a_quarter_sigma_on_unit_norm_rows():
    """The headline data: the slack (bound - exact) is ~0.008 on unit-norm d = 1024 rows — the number DESIGN §3.2
    quotes (a quarter of the score distribution's sigma, 1/32)."""
    rng = np.random.default_rng(0)
    x = rng.standard_normal((4000, 1024)).astype(F)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    v = rng.standard_normal(1024).astype(F)
    v /= np.linalg.norm(v)
    xq, sx, e = quantize_rows(x)
    u = bound(xq, sx, e, np.ones(len(x), F), *quantize_query(v))
    slack = u.astype(np.float64) - x.astype(np.float64) @ v.astype(np.float64)
    assert slack.min() >= 0
    assert 0.006 < np.median(slack) < 0.010


def test_one_piece_bound_on_unit_norm_bf16_rows():
    """DT 9 on config 5's data (unit-norm rows stored as bf16, one query piece): the bound holds and its slack stays
    within ~2x the two-piece screen's — the one-piece residual (up to 64x the two-piece one per element) adds
    eq |x| ~ 0.008 on unit-norm rows, next to the rows' own e (the 32-candidate verify proves it: profiles/r05)."""
    rng = np.random.default_rng(1)
    x = rng.standard_normal((4000, 1024)).astype(F)
    x = bf16_round(x / np.linalg.norm(x, axis=1, keepdims=True))
    v = rng.standard_normal(1024).astype(F)
    v /= np.linalg.norm(v)
    xq, sx, e = quantize_rows(x)
    nd = np.sqrt((x * x).sum(axis=1, dtype=F)).astype(F)
    u = bound(xq, sx, e, nd, *quantize_query(v, 1))
    slack = u.astype(np.float64) - x.astype(np.float64) @ v.astype(np.float64)
    assert slack.min() >= 0
    assert 0.008 < np.median(slack) < 0.02, float(np.median(slack))


def residual_aligned_row(v, b, target=0.5, pieces=1):
    """A row aligned with query v's quantisation residual r = v - scale (p1 [+ p2 / 64]): x = b r^
    + beta w (w: v's component orthogonal to r, beta so that x . v = target). Its x . r = b |r| is what the bound's
    eq |x| term carries — the int8 estimate cannot see it — so a bound fed a row norm of 1 instead of |x| ~ b misses it
    by ~eq (b - 1). Returns the row in float64."""
    p1, p2, qsc, _, _, _, w1 = quantize_query(v, pieces)
    approx = float(qsc) * (w1 * p1.astype(np.float64) + p2.astype(np.float64))
    r = v.astype(np.float64) - approx
    rh = r / np.linalg.norm(r)
    qp = v.astype(np.float64) - (v.astype(np.float64) @ rh) * rh
    w = qp / np.linalg.norm(qp)
    beta = (target - b * (v.astype(np.float64) @ rh)) / (w @ v.astype(np.float64))
    return b * rh + beta * w


@pytest.mark.parametrize("pieces", [1, 2])
def test_int8_bound_holds_on_residual_aligned_rows(pieces):
    """Rows aligned with the query's residual (the case random rows hide behind Cauchy-Schwarz slack): the bound with
    the rows' true norms holds at every scale; fed a norm of 1 (what bf16 + dot storage read before r6: its norms were
    never computed) it falls below the exact score once |x| is a few units — the hole the r6 fix closes."""
    rng = np.random.default_rng(42 + pieces)
    d = 1024
    v = rng.standard_normal(d).astype(F)
    v /= np.linalg.norm(v)
    bs = [1.0, 3.0, 10.0, 30.0, 100.0]
    x = np.stack([residual_aligned_row(v, b, pieces=pieces) for b in bs]).astype(F)
    if pieces == 1:
        x = bf16_round(x)
    xq, sx, e = quantize_rows(x)
    nd = np.sqrt((x * x).sum(axis=1, dtype=F)).astype(F)
    qv = quantize_query(v, pieces)
    exact = x.astype(np.float64) @ v.astype(np.float64)
    u = bound(xq, sx, e, nd, *qv).astype(np.float64)
    assert np.all(u >= exact), (u - exact)
    u1 = bound(xq, sx, e, np.ones_like(nd), *qv).astype(np.float64)
    if pieces == 1:   # one piece: the residual is ~64x the two-piece one, so the unit-norm bound fails from b ~ 10
        assert np.all(u1[2:] < exact[2:]), (u1 - exact)
