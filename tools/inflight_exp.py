"""In-process A/B of the async MSM stream at 2^20: serial vs k in flight,
with and without BPP_MSM_STAGGER, repeated to see box noise."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import bpperm  # noqa: E402

n = 1 << 20
if os.environ.get("WITH_TORCH") or os.environ.get("WITH_TORCH_LATE"):
    import torch
if os.environ.get("WITH_TORCH"):
    torch.cuda.synchronize()
ctx = bpperm.Context(0)
if os.environ.get("WITH_TORCH_LATE"):
    torch.cuda.synchronize()
pts = ctx.from_uniform(bench.synth_point_bytes(n, 3))
bufs = []
for seed in (2, 7):
    sc = bench.synth_scalars(n, seed)
    d = ctx.dev_alloc(len(sc))
    ctx.htod(d, sc)
    bufs.append(d)


def piped(k, steps):
    ticks, out = [], []
    for i in range(steps + k - 1):
        if i < steps:
            ticks.append(ctx.msm_submit(bufs[i % 2], pts, n))
        if i >= k - 1:
            out.append(ctx.msm_collect(ticks.pop(0)))
    return out


def serial(steps):
    return [ctx.msm_table_dev(bufs[i % 2], pts, n) for i in range(steps)]


for rep in range(int(os.environ.get("REPS", "2"))):
    for name, fn in [("serial", serial), ("k1", lambda s: piped(1, s)), ("k2", lambda s: piped(2, s)),
                     ("k3", lambda s: piped(3, s)), ("k2-stagger", lambda s: piped(2, s))]:
        if name.endswith("stagger"):
            os.environ["BPP_MSM_STAGGER"] = "1"
        fn(4)
        t = time.perf_counter()
        fn(20)
        el = (time.perf_counter() - t) / 20 * 1e3
        os.environ.pop("BPP_MSM_STAGGER", None)
        print(f"{name:12s} {el:.4f} ms/MSM", flush=True)
