"""Large-size MSM parity (the single-MSM sort paths, n >= 2^14: two-pass
radix sort by default, the one-pass LDS sort under BPP_MSM_LDS_SORT=1).

Exact: GPU vs the serial C restatement of dalek's MSM (oracle/c) at 2^14 and
2^17 terms.  Full size (BASELINE config 3, 2^20 terms): size-independent
properties — linearity in the scalars (MSM(s) + MSM(t) == MSM(s + t)),
window-partition consistency (sum of partials == full), and the adversarial
all-equal-scalar input (every term in one bucket per window)."""
import hashlib

import pytest

from bpperm._lib import BppError
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


@pytest.mark.parametrize("logn,lds,acc_k", [(14, False, None), (17, False, None), (17, True, None),
                                            (17, False, "12"), (14, False, "36"), (17, False, "100")])
def test_msm_exact_vs_cport(ctx, big_table, logn, lds, acc_k, monkeypatch):
    """acc_k: entries per accumulation lane forced to a non-power-of-two
    multiple of 4 (msm.hip picks one by size, e.g. 36 for config 5)."""
    if lds:
        monkeypatch.setenv("BPP_MSM_LDS_SORT", "1")
    if acc_k:
        monkeypatch.setenv("BPP_MSM_ACC_K", acc_k)
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


def test_msm_async_submit_collect(ctx, big_table):
    """bpp_msm_submit / bpp_msm_collect: two MSMs in flight give the same
    results as one at a time (collected out of order), window partials
    through the async path sum to the full MSM, one more than BPP_MSM_INFLIGHT outstanding submits
    is refused, and an unknown ticket is refused."""
    import bpperm
    from bpperm import dist as bdist
    raw, tbl = big_table
    n = 1 << 17
    sa, sb_ = _sb(_scalars(n, 31)), _sb(_scalars(n, 32))
    da, db = ctx.dev_alloc(32 * n), ctx.dev_alloc(32 * n)
    ctx.htod(da, sa)
    ctx.htod(db, sb_)
    want_a, want_b = ctx.msm_table_dev(da, tbl, n), ctx.msm_table_dev(db, tbl, n)
    assert want_a == cport.msm(sa, cport.from_uniform(raw[: 64 * n]))
    ta = ctx.msm_submit(da, tbl, n)
    tb = ctx.msm_submit(db, tbl, n)
    extra = [ctx.msm_submit(da, tbl, n) for _ in range(bpperm.MSM_INFLIGHT - 2)]
    with pytest.raises(BppError):
        ctx.msm_submit(da, tbl, n)
    assert ctx.msm_collect(tb) == want_b
    assert ctx.msm_collect(ta) == want_a
    assert all(ctx.msm_collect(t) == want_a for t in extra)
    with pytest.raises(BppError):
        ctx.msm_collect(ta)
    c, W = bpperm.msm_windows(n)
    parts = []
    for a, b in bdist.window_ranges(W, 3):
        parts.append(ctx.msm_collect(ctx.msm_submit(da, tbl, n, a, b), partial=True))
    assert bpperm.partials_finish(parts) == want_a
    # a long stream, two in flight, alternating inputs
    got, tick = [], ctx.msm_submit(da, tbl, n)
    for i in range(6):
        nxt = ctx.msm_submit(db if i % 2 == 0 else da, tbl, n) if i < 5 else None
        got.append(ctx.msm_collect(tick))
        tick = nxt
    assert got == [want_a, want_b] * 3
    ctx.dev_free(da)
    ctx.dev_free(db)


@pytest.mark.parametrize("up_streams", ["0", "2"])
def test_msm_submit_host_scalars(ctx, big_table, monkeypatch, up_streams):
    """bpp_msm_submit_host (host scalars, the reference's call shape): from
    pinned memory (the H2D copy on the MSM's own stream, or split over two
    upload streams the MSM's stream waits for: BPP_MSM_UP_STREAMS) and from
    pageable bytes (staged), several in flight, a window range; all equal the
    resident-scalar MSM and the C port."""
    import ctypes
    monkeypatch.setenv("BPP_MSM_UP_STREAMS", up_streams)

    import bpperm
    from bpperm import dist as bdist
    raw, tbl = big_table
    n = 1 << 17
    sa, sb_ = _sb(_scalars(n, 41)), _sb(_scalars(n, 42))
    want_a = cport.msm(sa, cport.from_uniform(raw[: 64 * n]))
    want_b = ctx.msm_table(sb_, tbl, n)
    ha, hb = ctx.host_alloc(32 * n), ctx.host_alloc(32 * n)
    ctypes.memmove(ha, sa, 32 * n)
    ctypes.memmove(hb, sb_, 32 * n)
    ticks = [ctx.msm_submit_host(ha, tbl, n), ctx.msm_submit_host(hb, tbl, n), ctx.msm_submit_host(sa, tbl, n)]
    assert [ctx.msm_collect(t) for t in ticks] == [want_a, want_b, want_a]
    c, W = bpperm.msm_windows(n)
    parts = [ctx.msm_collect(ctx.msm_submit_host(hb, tbl, n, a, b), partial=True) for a, b in bdist.window_ranges(W, 2)]
    assert bpperm.partials_finish(parts) == want_b
    ctx.host_free(ha)
    ctx.host_free(hb)


def test_msm_submit_host_noncanonical_scalars(ctx, big_table):
    """bpp_msm_submit_host does not check scalars for canonical
    form (bpp_msm_table does); a non-canonical host scalar gives exactly what
    bpp_msm_submit gives for the same bytes resident on the device -- pinned
    and pageable, across the pageable path's staging pieces.  For a value
    below 2^253 that is the MSM of the scalar reduced mod l (l * P is the
    identity of the ristretto group)."""
    import ctypes
    raw, tbl = big_table
    n = (1 << 17) + 5
    sc = _scalars(n, 43)
    sc[3] = L + 5          # non-canonical, < 2^253
    sc[n - 2] = 2 * L + 1  # non-canonical near the end (last staging piece)
    sb = _sb(sc)
    want = ctx.msm_table(_sb([s % L for s in sc]), tbl, n)
    d = ctx.dev_alloc(32 * n)
    h = ctx.host_alloc(32 * n)
    try:
        ctx.htod(d, sb)
        ctypes.memmove(h, sb, 32 * n)
        dev = ctx.msm_collect(ctx.msm_submit(d, tbl, n))
        pinned = ctx.msm_collect(ctx.msm_submit_host(h, tbl, n))
        pageable = ctx.msm_collect(ctx.msm_submit_host(sb, tbl, n))
        assert dev == pinned == pageable == want
        with pytest.raises(BppError):  # the one-at-a-time host entry point checks
            ctx.msm_table(sb, tbl, n)
    finally:
        ctx.dev_free(d)
        ctx.host_free(h)


def test_msm_2p22_config5_window_partition(ctx):
    """Config 5 shape (one 2^22-term batch-verify MSM, bucket windows
    partitioned over 8 GPUs), rehearsed on one GPU: the 8 ranks' window
    partials (bpp_msm_submit/collect, windows split as bpperm.dist does)
    sum to the full MSM, and the full MSM is linear in the scalars."""
    import bpperm
    from bpperm import dist as bdist
    n = 1 << 22
    raw = hashlib.shake_256(b"config5-points").digest(64 * n)
    tbl = ctx.from_uniform(raw)
    del raw
    # scalars < 2^252 < l (canonical): top nibble cleared
    sraw = bytearray(hashlib.shake_256(b"config5-scalars").digest(32 * n))
    sraw[31::32] = bytes(b & 0x0F for b in sraw[31::32])
    d = ctx.dev_alloc(32 * n)
    ctx.htod(d, bytes(sraw))
    full = ctx.msm_table_dev(d, tbl, n)
    c, W = bpperm.msm_windows(n)
    ranges = bdist.window_ranges(W, 8)
    parts = []
    for a, b in ranges:
        parts.append(ctx.msm_collect(ctx.msm_submit(d, tbl, n, a, b), partial=True))
    assert bpperm.partials_finish(parts) == full
    # linearity on the doubled scalars (2s < 2^253 < l stays canonical)
    import numpy as np
    a = np.frombuffer(bytes(sraw), dtype="<u8").reshape(n, 4)
    carry = np.concatenate([np.zeros((n, 1), dtype=np.uint64), a[:, :3] >> np.uint64(63)], axis=1)
    dbl = ((a << np.uint64(1)) | carry).astype("<u8").tobytes()
    ctx.htod(d, dbl)
    got2 = ctx.msm_table_dev(d, tbl, n)
    P = r255.decode(full)
    assert got2 == r255.encode(r255.ed_add(P, P))
    ctx.dev_free(d)
    tbl.close()


def _bench_inputs(ctx, world, seed_base=2):
    import bench
    n = 1 << 20
    tbl = ctx.from_uniform(b"".join(bench.synth_point_bytes(n, 3 + 1000 * s) for s in range(world)))
    sc = b"".join(bench.synth_scalars(n, seed_base + 1000 * s) for s in range(world))
    d = ctx.dev_alloc(len(sc))
    ctx.htod(d, sc)
    return tbl, d, world * n


def test_msm_2p20_exact_vs_cport_golden(ctx):
    """Config 3 at its full size, exact: the bench's own 2^20 inputs (both
    scalar vectors of its pipelined stream) against the C port's result
    (tests/golden/bench_msm.json, make_bench_golden.py), one MSM at a time
    and through the submit/collect stream bench.py times."""
    import json
    from pathlib import Path
    gold = json.loads((Path(__file__).parent / "golden" / "bench_msm.json").read_text())["world"]["1"]
    tbl, d, n = _bench_inputs(ctx, 1)
    assert ctx.msm_table_dev(d, tbl, n).hex() == gold["result"]
    import bench
    d2 = ctx.dev_alloc(32 * n)
    ctx.htod(d2, bench.synth_scalars(n, 7))
    t1 = ctx.msm_submit(d, tbl, n)
    t2 = ctx.msm_submit(d2, tbl, n)
    t3 = ctx.msm_submit(d, tbl, n)
    assert ctx.msm_collect(t1).hex() == gold["result"]
    assert ctx.msm_collect(t2).hex() == gold["result2"]
    assert ctx.msm_collect(t3).hex() == gold["result"]
    ctx.dev_free(d)
    ctx.dev_free(d2)
    tbl.close()


def test_msm_2p21_both_partitions_exact(ctx):
    """bench.py at N = 2, rehearsed on one GPU: the window split (each rank
    all 2^21 points, half the windows) and the point split (each rank its
    2^20-point slice, all windows) both reproduce the C port's 2^21 result
    after the exact partial addition (bpp_partials_finish)."""
    import json
    from pathlib import Path

    import bpperm
    from bpperm import dist as bdist
    gold = json.loads((Path(__file__).parent / "golden" / "bench_msm.json").read_text())["world"]["2"]
    tbl, d, n = _bench_inputs(ctx, 2)
    c, W = bpperm.msm_windows(n)
    parts = [ctx.msm_table_dev_partial(d, tbl, n, a, b) for a, b in bdist.window_ranges(W, 2)]
    assert bpperm.partials_finish(parts).hex() == gold["result"]
    tbl.close()
    ctx.dev_free(d)
    import bench
    half = 1 << 20
    parts = []
    for s in range(2):
        t = ctx.from_uniform(bench.synth_point_bytes(half, 3 + 1000 * s))
        ds = ctx.dev_alloc(32 * half)
        ctx.htod(ds, bench.synth_scalars(half, 2 + 1000 * s))
        _, Wh = bpperm.msm_windows(half)
        parts.append(ctx.msm_table_dev_partial(ds, t, half, 0, Wh))
        ctx.dev_free(ds)
        t.close()
    assert bpperm.partials_finish(parts).hex() == gold["result"]


def test_msm_2p22_exact_vs_cport_golden_window_partition(ctx):
    """Config 5 as BASELINE.json states it (one 2^22-term MSM, bucket windows
    partitioned over 8 GPUs), exact: bench.py's msm_2e22 inputs (its four
    2^20 slices) against the C port's result (tests/golden/bench_msm.json
    world 4): the whole MSM one at a time and through the submit/collect
    stream, and the 8 window-range partials (as bpperm.dist splits them for
    8 ranks) added exactly (bpp_partials_finish)."""
    import json
    from pathlib import Path

    import bpperm
    from bpperm import dist as bdist
    gold = json.loads((Path(__file__).parent / "golden" / "bench_msm.json").read_text())["world"]["4"]
    tbl, d, n = _bench_inputs(ctx, 4)
    assert n == 1 << 22
    assert ctx.msm_table_dev(d, tbl, n).hex() == gold["result"]
    assert ctx.msm_collect(ctx.msm_submit(d, tbl, n)).hex() == gold["result"]
    c, W = bpperm.msm_windows(n)
    parts = [ctx.msm_collect(ctx.msm_submit(d, tbl, n, a, b), partial=True) for a, b in bdist.window_ranges(W, 8)]
    assert bpperm.partials_finish(parts).hex() == gold["result"]
    ctx.dev_free(d)
    tbl.close()


def test_host_scalar_upload_pieces_and_bad_index(ctx, big_table):
    """Host scalars are staged, checked and copied in 4-MB pieces (131072
    scalars, msm.hip upload_scalars): a 2^18 + 5-term MSM crosses two piece
    borders and equals the same MSM over device-resident scalars; a
    non-canonical scalar in the third piece fails the call with its index."""
    _, tbl = big_table
    n = (1 << 18) + 5
    sb = _sb(_scalars(n, 18))
    d = ctx.dev_alloc(32 * n)
    ctx.htod(d, sb)
    assert ctx.msm_table(sb, tbl, n) == ctx.msm_table_dev(d, tbl, n)
    ctx.dev_free(d)
    bad = 2 * 131072 + 3
    sb2 = sb[: 32 * bad] + L.to_bytes(32, "little") + sb[32 * bad + 32:]
    with pytest.raises(BppError) as ei:
        ctx.msm_table(sb2, tbl, n)
    assert ei.value.name == "BPP_ERR_NONCANONICAL"
    assert f"index {bad}" in str(ei.value)
