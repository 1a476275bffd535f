"""Experiment: does splitting one 2^20 MSM's windows over 2 / 4 streams
(child contexts driven from host threads) overlap the latency-bound tails
(bucket reduction) of one group with the accumulation of another?"""
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))
import bpperm  # noqa: E402
import bench  # noqa: E402

n = 1 << 20
ctxs = [bpperm.Context(0) for _ in range(5)]
c0 = ctxs[0]
pts = c0.from_uniform(bench.synth_point_bytes(n, 3))
sc = bench.synth_scalars(n, 2)
d = c0.dev_alloc(len(sc))
c0.htod(d, sc)
c, W = bpperm.msm_windows(n)
ref = c0.msm_table_dev(d, pts, n)


def split_run(k):
    cuts = [W * i // k for i in range(k + 1)]
    parts = [None] * k

    def work(i):
        parts[i] = ctxs[1 + i].msm_table_dev_partial(d, pts, n, cuts[i], cuts[i + 1])

    th = [threading.Thread(target=work, args=(i,)) for i in range(k)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return bpperm.partials_finish(parts)


for k in (1, 2, 4):
    res = split_run(k) if k > 1 else c0.msm_table_dev(d, pts, n)
    assert res == ref, k
    t = time.perf_counter()
    for _ in range(10):
        res = split_run(k) if k > 1 else c0.msm_table_dev(d, pts, n)
    dt = (time.perf_counter() - t) / 10
    print(f"streams={k}: {dt * 1e3:.3f} ms per 2^20 MSM -> {n / dt / 1e6:.1f} M pairs/s")
