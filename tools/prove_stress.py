"""Host-fault hunt for the prover's production entry point: entropy batches
of varying sizes interleaved with u64-seed batches on one context, for a
bounded time, every result verified.  Run with BPP_SEGV_TRACE=1 so a fault
prints libbpperm's native backtrace.
    python tools/prove_stress.py [seconds]"""
import os
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
import bpperm  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
    rnd = random.Random(7)
    ctx = bpperm.Context(0)
    g = bpperm.Gens(ctx, 128)
    provers = {k: bpperm.PermProver(g, k) for k in (4, 5, 52)}
    t0, n, it = time.time(), 0, 0
    while time.time() - t0 < secs:
        k = rnd.choice((4, 5, 52))
        pr = provers[k]
        cnt = rnd.choice((1, 3, 9, 17, 41, 64))
        if rnd.random() < 0.5:
            proofs, Vs = pr.prove_batch_entropy(cnt, os.urandom(32 * cnt) if rnd.random() < 0.5 else None)
        else:
            proofs, Vs = pr.prove_batch([rnd.randrange(1 << 62) for _ in range(cnt)])
        assert pr.verify_batch(proofs, Vs), (k, cnt)
        n += cnt
        it += 1
    print("ok", it, "batches", n, "proofs")


if __name__ == "__main__":
    main()
