"""Per-stage times of one batch verification (config 5 shape by default):
the host phases and the device kernels (HIP events), averaged over --reps
verifications after one warm run.  BPP_LIB selects an A/B build
(build.py --variant ... -D EXP_...; timing-only variants verify False).

    python tools/verify_stages.py [--proofs 4096] [--reps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

STAGES = ("verify_upload", "verify_replay", "verify_terms", "verify_replay_dev", "verify_replay_post", "verify_decompress",
          "verify_scalars", "msm_digits", "msm_scatter", "msm_accumulate", "msm_reduce")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=52)
    ap.add_argument("--pinned", action="store_true", help="the last (traced) verification from pinned host buffers")
    a = ap.parse_args()
    import bpperm
    ctx = bpperm.Context(0)
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, a.k)
    proofs, Vs = [], []
    for b in range(0, a.proofs, 256):
        p, v = pr.prove_batch(list(range(900_000 + b, 900_000 + min(a.proofs, b + 256))))
        proofs += p
        Vs += v
    proofs, Vs = b"".join(proofs), b"".join(Vs)  # (contiguous, as bench.py passes them)
    ok = pr.verify_batch(proofs, Vs)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        pr.verify_batch(proofs, Vs)
    wall = (time.perf_counter() - t0) / a.reps * 1e3
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(a.reps):
        pr.verify_batch(proofs, Vs)
    st = {s: round(ctx.profile_get(s)[0] / a.reps, 4) for s in STAGES}
    ctx.profile(False)
    # one unprofiled verification last: tools/verify_timeline.py reads the
    # last batch of a trace, and the stage scopes' events would add gaps
    if a.pinned:
        import ctypes
        hp, hv = ctx.host_alloc(len(proofs)), ctx.host_alloc(len(Vs))
        ctypes.memmove(hp, proofs, len(proofs))
        ctypes.memmove(hv, Vs, len(Vs))
        pr.verify_batch_ptr(hp, hv, a.proofs)
        t0 = time.perf_counter()
        pr.verify_batch_ptr(hp, hv, a.proofs)
        last = (time.perf_counter() - t0) * 1e3
    else:
        pr.verify_batch(proofs, Vs)
        t0 = time.perf_counter()
        pr.verify_batch(proofs, Vs)
        last = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"last_ms": round(last, 4), "pinned": a.pinned, "proofs": a.proofs, "verified": ok, "wall_ms": round(wall, 4),
                      "proofs_per_s": a.proofs / wall * 1e3, "stage_ms": st}))
    if a.pinned:
        ctx.host_free(hp)
        ctx.host_free(hv)
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
