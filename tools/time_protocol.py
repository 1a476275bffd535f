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
for B, S in ((16, "1"), (128, "1"), (256, "1"), (512, "1")):
    os.environ["BPP_PROVE_STREAMS"] = S
    print(f"-- streams {S}")
    pr.prove_batch(list(range(B)))
    tp, tv = [], []
    for rep in range(3):
        t = time.perf_counter()
        proofs, Vs = pr.prove_batch(list(range(1000 * (rep + 1), 1000 * (rep + 1) + B)))
        tp.append(time.perf_counter() - t)
        t = time.perf_counter()
        assert pr.verify_batch(proofs, Vs)
        tv.append(time.perf_counter() - t)
    print(f"prove_batch {B}: {[round(x * 1e3, 2) for x in tp]} ms  -> {B / min(tp):.0f} proofs/s (best)")
    print(f"verify_batch {B}: {[round(x * 1e3, 2) for x in tv]} ms  -> {B / min(tv):.0f} proofs/s (best)")
for S, B in (("1", 128), ("1", 512), ("2", 512)):
    os.environ["BPP_PROVE_STREAMS"] = S
    pr.prove_batch(list(range(B)))
    ctx.profile(True)
    ctx.profile_reset()
    t = time.perf_counter()
    pr.prove_batch(list(range(B)))
    print(f"profile of prove_batch({B}), streams {S}: wall {(time.perf_counter() - t) * 1e3:.2f} ms")
    for st in ("pedersen", "msm_count", "msm_scatter", "msm_accumulate", "msm_fixup", "msm_reduce", "msm_scan",
               "compress", "ipa_terms", "ipa_fold", "ipa_msm", "ipa_host", "pb_rng", "pb_pedersen_V",
               "pb_pedersen_Vx_witness", "pb_msm_AI_AO_S", "pb_host_poly", "pb_pedersen_T_lr", "pb_ipa"):
        ms, k = ctx.profile_get(st)
        print(f"  {st:22s} {ms:8.3f} ms over {k} launches")
    ctx.profile(False)
