"""One rank's share of an N-GPU weak-scaling MSM run, timed on ONE GPU.

bench.py --gpus N (window split, the default) gives every rank all
N * 2^log2n points and W/N of the W bucket windows; the point split gives it
its own 2^log2n points and all W windows (= the N=1 work).  This runs rank
r's window-split share alone on the card (no collective: the partial point
is collected raw), so the per-rank cost at N = 2, 4, 8 can be seen before the
driver's multi-GPU run: larger point tables (2^23 x 128 B = 1 GB at N = 8)
leave the 256 MB Infinity Cache, and fewer windows per rank leave the bucket
reduction with fewer waves.

    python tools/rank_share.py [N ...] [--log2n 20] [--steps 10]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))
import bpperm  # noqa: E402
from bench import synth_point_bytes, synth_scalars  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ns", type=int, nargs="*", default=[2, 4, 8])
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=2)
    args = ap.parse_args()
    n_local = 1 << args.log2n
    ctx = bpperm.Context(0)
    for N in args.ns:
        n = n_local * N
        pts = ctx.from_uniform(b"".join(synth_point_bytes(n_local, 3 + 1000 * s) for s in range(N)))
        bufs = []
        for seed in (2, 7):
            sc = b"".join(synth_scalars(n_local, seed + 1000 * s) for s in range(N))
            d = ctx.dev_alloc(len(sc))
            ctx.htod(d, sc)
            bufs.append(d)
        c, W = bpperm.msm_windows(n)
        cuts = [(W * r) // N for r in range(N + 1)]
        for r in sorted({0, N - 1}):
            wb, we = cuts[r], cuts[r + 1]

            def stream(k):
                ticks = []
                for i in range(k + args.inflight - 1):
                    if i < k:
                        ticks.append(ctx.msm_submit(bufs[i % 2], pts, n, wb, we))
                    if i >= args.inflight - 1:
                        ctx.msm_collect(ticks.pop(0), partial=True)

            stream(max(args.steps, 8))  # warm the child contexts
            t0 = time.perf_counter()
            stream(args.steps)
            el = (time.perf_counter() - t0) / args.steps
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ctx.msm_table_dev_partial(bufs[0], pts, n, wb, we)
            lat = (time.perf_counter() - t0) / args.steps
            ctx.profile(True)
            ctx.profile_reset()
            for _ in range(3):
                ctx.msm_table_dev_partial(bufs[0], pts, n, wb, we)
            stages = {}
            for st in ("msm_digits", "msm_scan", "msm_scatter", "msm_accumulate", "msm_fixup", "msm_reduce"):
                ms, k = ctx.profile_get(st)
                stages[st] = round(ms / 3, 4)
            ctx.profile(False)
            row = {"n_gpus": N, "rank": r, "pairs": n, "windows": [wb, we], "window_bits": c,
                   "ms_per_msm_pipelined": el * 1e3, "ms_per_msm_one_at_a_time": lat * 1e3,
                   "projected_pairs_per_s_whole_job": n / el, "stage_ms": stages}
            print(json.dumps(row), flush=True)
        for d in bufs:
            ctx.dev_free(d)
        pts.close()
    ctx.close()


if __name__ == "__main__":
    main()
