"""Config 2 (2^10 vector commitment + IPA) one at a time, for a kernel /
memory-copy trace (rocprofv3 ... -- python3 tools/config2_once.py [reps]):
bench.py's own bench_config2 with a wall-clock timer.

    python tools/config2_once.py 5
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))


def main():
    import bench
    import bpperm
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5

    def timed(fn):
        t0 = time.perf_counter()
        out = fn()
        return out, time.perf_counter() - t0

    ctx = bpperm.Context(0)
    r = bench.bench_config2(ctx, timed, reps=reps)
    print(r["latency_ms"], r["result_ok"])
    ctx.close()


if __name__ == "__main__":
    main()
