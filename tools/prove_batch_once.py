"""One warm prove_batch + verify_batch of B 52-card proofs (for rocprofv3
kernel traces of the batched prover)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
import bpperm  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx = bpperm.Context(0)
g = bpperm.Gens(ctx, 128)
pr = bpperm.PermProver(g, 52)
pr.prove_batch(list(range(B)))
for rep in range(3):
    proofs, Vs = pr.prove_batch(list(range(B * (rep + 1), B * (rep + 2))))
    ok = pr.verify_batch(proofs, Vs)
    assert ok or os.environ.get("BPP_LIB"), "proofs must verify (timing-only variants excepted)"
print("ok")
