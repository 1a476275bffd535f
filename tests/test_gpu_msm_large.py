"""Large-size MSM parity (the single-MSM sort paths, n >= 2^14: two-pass
radix sort by default, the one-pass LDS sort under BPP_MSM_LDS_SORT=1).

Exact: GPU vs the serial C restatement of dalek's MSM (oracle/c) at 2^14 and
2^17 terms.  Full size (BASELINE config 3, 2^20 terms): size-independent
properties — linearity in the scalars (MSM(s) + MSM(t) == MSM(s + t)),
window-partition consistency (sum of partials == full), and the adversarial
all-equal-scalar input (every term in one bucket per window)."""
import hashlib

import pytest

from oracle import cport, ristretto as r255

pytestmark = pytest.mark.gpu
L = r255.L


def _scalars(n, seed):
    raw = hashlib.shake_256(b"large-msm" + seed.to_bytes(8, "little")).digest(64 * n)
    return [int.from_bytes(raw[64 * i: 64 * i + 64], "little") % L for i in range(n)]


def _sb(sc):
    return b"".join(s.to_bytes(32, "little") for s in sc)


@pytest.fixture(scope="module")
def big_table(ctx):
    raw = hashlib.shake_256(b"large-msm-points").digest(64 * (1 << 20))
    t = ctx.from_uniform(raw)
    yield raw, t
    t.close()


@pytest.mark.parametrize("logn,lds", [(14, False), (17, False), (17, True)])
def test_msm_exact_vs_cport(ctx, big_table, logn, lds, monkeypatch):
    if lds:
        monkeypatch.setenv("BPP_MSM_LDS_SORT", "1")
    raw, tbl = big_table
    n = 1 << logn
    sc = _sb(_scalars(n, logn))
    pts = cport.from_uniform(raw[: 64 * n])
    assert ctx.msm_table(sc, tbl, n) == cport.msm(sc, pts)


def test_msm_2p20_linearity_and_partials(ctx, big_table):
    import bpperm
    from bpperm import dist as bdist
    _, tbl = big_table
    n = 1 << 20
    s = _scalars(n, 1)
    t = _scalars(n, 2)
    u = [(a + b) % L for a, b in zip(s, t)]
    ms, mt, mu = (ctx.msm_table(_sb(x), tbl, n) for x in (s, t, u))
    lhs = r255.ed_add(r255.decode(ms), r255.decode(mt))
    assert r255.encode(lhs) == mu
    d = ctx.dev_alloc(32 * n)
    ctx.htod(d, _sb(s))
    c, W = bpperm.msm_windows(n)
    parts = [ctx.msm_table_dev_partial(d, tbl, n, a, b) for a, b in bdist.window_ranges(W, 3)]
    assert bpperm.partials_finish(parts) == ms
    ctx.dev_free(d)


@pytest.mark.parametrize("n", [1 << 16, 1 << 20])
def test_msm_all_equal_scalars(ctx, big_table, n):
    """Adversarial bucket skew: n equal scalars put every term of a window in
    one bucket (one coarse bin of 2^20 entries: the multi-tile fine sort, and
    2^14 accumulate chunks for fixup to join); sum_i k P_i == k * sum_i P_i."""
    _, tbl = big_table
    k = _scalars(1, 9)[0]
    got = ctx.msm_table(_sb([k] * n), tbl, n)
    ones = ctx.msm_table(_sb([1] * n), tbl, n)
    assert got == r255.encode(r255.ed_mul(k, r255.decode(ones)))
