"""Config 2's host phases: bench.py's bench_config2 flow with the library's
host scopes on (ms per run: the IPA's waits, double encodings, transcript
and challenge inversions) and the Python-side steps timed around it.

    python tools/config2_phases.py [reps]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

STAGES = ["ipa_wait", "ipa_msm", "double_encode", "ipa_host", "ipa_uinv", "ipa_round_dt"]


def main():
    import bench
    import bpperm
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ctx = bpperm.Context(0)

    def timed(fn):
        t0 = time.perf_counter()
        out = fn()
        return out, time.perf_counter() - t0

    r = bench.bench_config2(ctx, timed, reps=reps)
    print("plain %.4f ms ok %s" % (r["latency_ms"], r["result_ok"]))
    ctx.profile(True)
    ctx.profile_reset()
    r = bench.bench_config2(ctx, timed, reps=reps)
    print("profiled %.4f ms ok %s" % (r["latency_ms"], r["result_ok"]))
    for s in STAGES:
        try:
            ms, n = ctx.profile_get(s)
        except Exception:
            continue
        print("  %-14s %8.4f ms per run (%d calls)" % (s, ms / (reps + 1), n))
    # the caller-side steps of one run (Python + ctypes)
    y = bpperm.Transcript(b"x").challenge_scalar(b"y")
    t0 = time.perf_counter()
    for _ in range(200):
        yi = bpperm.scalar_invert(y)
    t1 = time.perf_counter()
    for _ in range(200):
        bpperm.scalar_powers(yi, 1024)
    t2 = time.perf_counter()
    print("  scalar_invert %.1f us, scalar_powers(1024) %.1f us" % ((t1 - t0) / 200 * 1e6, (t2 - t1) / 200 * 1e6))
    ctx.close()


if __name__ == "__main__":
    main()
