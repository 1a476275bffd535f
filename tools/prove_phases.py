"""Per-phase wall times of the batched prover (HostScope / ProfScope stages,
ms per batch) and the plain batch time, for B proofs per batch.

    python tools/prove_phases.py [B] [reps]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
import bpperm  # noqa: E402

STAGES = ["pb_rng", "pb_pedersen_V", "pb_pedersen_Vx_witness", "pb_msm_AI_AO_S", "pb_host_poly",
          "pb_pedersen_T_lr", "pbT_pedersen", "pbT_host", "pb_ipa", "ipa_host", "ipa_msm", "ipa_terms",
          "ipa_fold", "pedersen", "ped_upload", "ped_kernels", "ped_d2h", "msm_direct", "ipa_round_dt", "double_encode",
          "compress", "poly_coef", "poly_x"]

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx = bpperm.Context(0)
g = bpperm.Gens(ctx, 128)
pr = bpperm.PermProver(g, 52)
pr.prove_batch(list(range(B)))
pr.prove_batch(list(range(B, 2 * B)))
t = time.perf_counter()
for r in range(reps):
    pr.prove_batch(list(range(B * (r + 2), B * (r + 3))))
plain = (time.perf_counter() - t) / reps * 1e3
ctx.profile(True)
ctx.profile_reset()
t = time.perf_counter()
for r in range(reps):
    pr.prove_batch(list(range(B * (r + 2), B * (r + 3))))
prof = (time.perf_counter() - t) / reps * 1e3
print(f"B={B}: {plain:.3f} ms/batch plain ({B / plain * 1e3:.0f} proofs/s), {prof:.3f} ms/batch profiled")
for s in STAGES:
    try:
        ms, n = ctx.profile_get(s)
    except Exception:
        continue
    if n:
        print(f"  {s:24s} {ms / reps:8.3f} ms/batch  ({n / reps:.1f} calls)")
