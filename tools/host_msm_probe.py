"""Host-scalar MSM stream probe: per-call host time of bpp_msm_submit_host and
bpp_msm_collect (does the submit block on the upload?), for pinned zero copy,
pinned + copy (BPP_MSM_HOST_COPY=1) and pageable bytes, 2^20 pairs, 3 in
flight.   python tools/host_msm_probe.py
(BPP_MSM_UP_CACHED=1: the upload buffer as an ordinary cached allocation)"""
import ctypes
import hashlib
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (synthetic inputs)


def main():
    import bpperm
    n = 1 << 20
    ctx = bpperm.Context(0)
    pts = ctx.from_uniform(bench.synth_point_bytes(n, 3))
    sc = [bench.synth_scalars(n, 2), bench.synth_scalars(n, 7)]
    hb = [ctx.host_alloc(32 * n) for _ in sc]
    for h, x in zip(hb, sc):
        ctypes.memmove(h, x, 32 * n)
    d = [ctx.dev_alloc(32 * n) for _ in sc]
    for p, x in zip(d, sc):
        ctx.htod(p, x)
    for mode in ("resident", "pinned", "pageable"):

        def sub(i):
            if mode == "resident":
                return ctx.msm_submit(d[i % 2], pts, n)
            return ctx.msm_submit_host(hb[i % 2] if mode.startswith("pinned") else sc[i % 2], pts, n)

        for rep in range(2):
            ts, tc, ticks = [], [], []
            t0 = time.perf_counter()
            K = 30
            for i in range(K + 2):
                if i < K:
                    a = time.perf_counter()
                    ticks.append(sub(i))
                    ts.append(time.perf_counter() - a)
                if i >= 2:
                    a = time.perf_counter()
                    ctx.msm_collect(ticks.pop(0))
                    tc.append(time.perf_counter() - a)
            el = time.perf_counter() - t0
        print(f"{mode:12s} {el / K * 1e3:.3f} ms/MSM  submit {sum(ts) / len(ts) * 1e3:.3f} ms  "
              f"collect {sum(tc) / len(tc) * 1e3:.3f} ms", flush=True)
    for h in hb:
        ctx.host_free(h)


if __name__ == "__main__":
    main()
