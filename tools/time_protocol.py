"""Time the protocol paths on one GPU (52-card proof, verify, batch verify,
2^10 commit + IPA) with the library's per-stage profile."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
sys.path.insert(0, str(ROOT))
import bpperm  # noqa: E402

import os  # noqa: E402

ctx = bpperm.Context(0)
g = bpperm.Gens(ctx, 1024)
pr = bpperm.PermProver(g, 52)
for mode in ("0", "1", None):
    if mode is None:
        os.environ.pop("BPP_MSM_FB", None)
    else:
        os.environ["BPP_MSM_FB"] = mode
    print(f"-- BPP_MSM_FB={mode}")
    pr.prove(0)
    t = time.perf_counter()
    N = 20
    for s in range(N):
        proof, V, _ = pr.prove(s)
    print(f"52-card prove: {(time.perf_counter() - t) / N * 1e3:.2f} ms/proof")
    t = time.perf_counter()
    for s in range(N):
        assert pr.verify(proof, V)
    print(f"52-card verify: {(time.perf_counter() - t) / N * 1e3:.2f} ms/proof")
    proofs, Vs = pr.prove_batch(list(range(64)))
    t = time.perf_counter()
    assert pr.verify_batch(proofs, Vs)
    print(f"batch verify 64: {(time.perf_counter() - t) * 1e3:.2f} ms total")
os.environ.pop("BPP_MSM_FB", None)
for B in (16, 128, 512):
    pr.prove_batch(list(range(B)))
    t = time.perf_counter()
    proofs, Vs = pr.prove_batch(list(range(1000, 1000 + B)))
    dt = time.perf_counter() - t
    print(f"prove_batch {B}: {dt * 1e3:.2f} ms  -> {B / dt:.0f} proofs/s")
    t = time.perf_counter()
    assert pr.verify_batch(proofs, Vs)
    dt = time.perf_counter() - t
    print(f"verify_batch {B}: {dt * 1e3:.2f} ms  -> {B / dt:.0f} proofs/s")
ctx.profile(True)
ctx.profile_reset()
pr.prove_batch(list(range(128)))
print("profile of prove_batch(128):")
for st in ("fbw_tables", "pedersen", "msm_count", "msm_scatter", "msm_accumulate", "msm_fixup", "msm_reduce",
           "msm_scan", "msm_horner", "compress", "ipa_terms", "ipa_fold"):
    ms, k = ctx.profile_get(st)
    print(f"  {st:16s} {ms:8.3f} ms over {k} launches")
ctx.profile(True)
ctx.profile_reset()
pr.prove(1)
for st in ("fbw_tables", "pedersen", "msm_count", "msm_scatter", "msm_accumulate", "msm_fixup", "msm_reduce", "msm_scan",
           "msm_horner", "ipa_terms", "ipa_fold"):
    ms, k = ctx.profile_get(st)
    print(f"  {st:16s} {ms:8.3f} ms over {k} launches")
ctx.profile(False)
