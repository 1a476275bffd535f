"""prove_batch phase profile for one batch size under the current
BPP_HOST_THREADS / BPP_PROVE_STREAMS (run once per setting)."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
import bpperm  # noqa: E402

B = int(sys.argv[1])
ctx = bpperm.Context(0)
g = bpperm.Gens(ctx, 128)
pr = bpperm.PermProver(g, 52)
pr.prove_batch(list(range(B)))
ts = []
for rep in range(3):
    t = time.perf_counter()
    pr.prove_batch(list(range(B * (rep + 1), B * (rep + 2))))
    ts.append(round((time.perf_counter() - t) * 1e3, 2))
ctx.profile(True)
ctx.profile_reset()
t = time.perf_counter()
pr.prove_batch(list(range(B)))
w = (time.perf_counter() - t) * 1e3
print(f"B={B} threads={os.environ.get('BPP_HOST_THREADS')} streams={os.environ.get('BPP_PROVE_STREAMS')} "
      f"reps={ts} profiled wall={w:.2f} ms")
for st in ("pb_rng", "pb_pedersen_V", "pb_pedersen_Vx_witness", "pb_msm_AI_AO_S", "pb_host_poly", "pbT_pedersen",
           "pbT_host", "pb_ipa", "ipa_msm", "ipa_host", "ped_upload", "ped_kernels", "ped_d2h", "pedersen",
           "compress", "msm_direct", "double_encode", "poly_coef", "poly_x"):
    ms, k = ctx.profile_get(st)
    print(f"  {st:22s} {ms:8.3f} ms over {k}")
