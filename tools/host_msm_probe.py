"""Host-scalar MSM stream probe: per-call host time of bpp_msm_submit_host and
bpp_msm_collect for resident, pinned and pageable scalars, 2^20 pairs, 3 in
flight; "dma alone" times the 32 MB H2D copy by itself and "resident+dma"
runs an unrelated copy per MSM on a stream of its own beside the resident
stream.   python tools/host_msm_probe.py [modes..]
UPS="0 1 2" REPS=3 K=60: each mode per BPP_MSM_UP_STREAMS value, interleaved."""
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
    hip = ctypes.CDLL("libamdhip64.so")
    strm = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(strm)) == 0
    scratch = ctx.dev_alloc(32 * n)

    def dma(i):  # an unrelated 32 B x n H2D copy on its own stream
        assert hip.hipMemcpyAsync(ctypes.c_void_p(scratch), ctypes.c_void_p(hb[i % 2]), ctypes.c_size_t(32 * n),
                                  1, strm) == 0

    for rep in range(2):  # the copies alone
        t0 = time.perf_counter()
        for i in range(30):
            dma(i)
        hip.hipStreamSynchronize(strm)
        print(f"dma alone    {(time.perf_counter() - t0) / 30 * 1e3:.3f} ms/copy", flush=True)
    modes = sys.argv[1:] or ["resident", "resident+dma", "pinned", "pageable"]
    # UPS="0 1 2": each mode once per BPP_MSM_UP_STREAMS value, interleaved
    # over REPS passes (the library reads the variable on every submit)
    ups = os.environ.get("UPS", "").split() or [None]
    runs = [(u, m) for _ in range(int(os.environ.get("REPS", "1"))) for u in ups for m in modes]
    K = int(os.environ.get("K", "30"))
    for up, mode in runs:
        if up is not None:
            os.environ["BPP_MSM_UP_STREAMS"] = up

        def sub(i):
            if mode == "resident+dma":
                dma(i)
            if mode.startswith("resident"):
                return ctx.msm_submit(d[i % 2], pts, n)
            return ctx.msm_submit_host(hb[i % 2] if mode.startswith("pinned") else sc[i % 2], pts, n)

        for rep in range(2):
            ts, tc, ticks = [], [], []
            t0 = time.perf_counter()
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
        print(f"up={up} {mode:12s} {el / K * 1e3:.3f} ms/MSM  submit {sum(ts) / len(ts) * 1e3:.3f} ms  "
              f"collect {sum(tc) / len(tc) * 1e3:.3f} ms", flush=True)
    for h in hb:
        ctx.host_free(h)


if __name__ == "__main__":
    main()
