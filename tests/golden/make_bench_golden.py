"""Expected results of bench.py's MSM workload, from the CPU port.

    python tests/golden/make_bench_golden.py [--log2n 20] [--slices 8]

bench.py's MSM at N ranks (either partition) is the MSM over the
concatenation of slices s = 0..N-1, slice s being 2^log2n points
from_uniform_bytes(SHAKE256("bench-points" || 3 + 1000 s)) and scalars
synth_scalars(2^log2n, 2 + 1000 s) -- or, for the second scalar vector the
pipelined stream alternates with, synth_scalars(2^log2n, 7 + 1000 s).  Each
slice is computed once with the serial C restatement of dalek's MSM
(oracle/c/dalek_port.c) on all host cores (oracle.cport.msm_threads), and
the per-N results are the prefix sums over slices, added with the Python
spec oracle.  Output: tests/golden/bench_msm.json, read by bench.py (its
`result_ok` field) and tests/test_gpu_msm_large.py (exact full-size check).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (synth_scalars / synth_point_bytes: the bench's own inputs)
from oracle import cport, ristretto as r255  # noqa: E402


def slice_results(log2n: int, s: int):
    n = 1 << log2n
    pts = cport.from_uniform_threads(bench.synth_point_bytes(n, 3 + 1000 * s))
    a = cport.msm_threads(bench.synth_scalars(n, 2 + 1000 * s), pts)
    b = cport.msm_threads(bench.synth_scalars(n, 7 + 1000 * s), pts)
    return a, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--slices", type=int, default=8)
    args = ap.parse_args()
    t0 = time.time()
    acc = [r255.IDENTITY, r255.IDENTITY]
    out = {"generator": "tests/golden/make_bench_golden.py (oracle/c/dalek_port.c on all host cores)",
           "log2n": args.log2n, "world": {}}
    for s in range(args.slices):
        a, b = slice_results(args.log2n, s)
        acc = [r255.ed_add(acc[0], r255.decode(a)), r255.ed_add(acc[1], r255.decode(b))]
        world = s + 1
        if world & (world - 1) == 0:  # N = 1, 2, 4, 8
            out["world"][str(world)] = {"result": r255.encode(acc[0]).hex(), "result2": r255.encode(acc[1]).hex()}
        print(f"slice {s}: {time.time() - t0:.1f} s", flush=True)
    out["seconds"] = round(time.time() - t0, 1)
    (HERE / "bench_msm.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
