"""Phase times of k_verify_scalars (one workgroup per proof) from the timing
variant's clock stamps: build it with
    python bulletproof-perm_amd/build.py --variant vst -D VS_TIMING
and run with BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_vst.so
    python tools/vs_phases.py [--proofs 4096]
Prints, over the batch's workgroups, the median cycles of each phase and the
spread of the workgroups' start times (how many rounds the grid took)."""
import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

PHASES = ["records+tables", "gate loop", "z^q c", "V_j columns", "A..R_j scalars", "block sums", "final lane 0"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=4096)
    a = ap.parse_args()
    import numpy as np

    import bpperm
    from bpperm import _lib
    lib = _lib.load()
    ctx = bpperm.Context(0)
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, 52)
    proofs, Vs = [], []
    for b in range(0, a.proofs, 256):
        p, v = pr.prove_batch(list(range(900_000 + b, 900_000 + min(a.proofs, b + 256))))
        proofs += p
        Vs += v
    pb, vb = b"".join(proofs), b"".join(Vs)
    pr.verify_batch(pb, vb)
    ok = pr.verify_batch(pb, vb)
    n = min(a.proofs, 8192)
    buf = (ctypes.c_ulonglong * (n * 8))()
    fn = lib.bpp_debug_vs_timing
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf, n * 8) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)
    d = np.diff(t, axis=1)
    start = t[:, 0] - t[:, 0].min()
    out = {"verified": ok, "median_cycles": {ph: int(np.median(d[:, i])) for i, ph in enumerate(PHASES)},
           "median_total": int(np.median(t[:, 7] - t[:, 0])),
           "start_spread_cycles": {q: int(np.percentile(start, q)) for q in (0, 25, 50, 75, 100)},
           "end_max_cycles": int((t[:, 7] - t[:, 0].min()).max())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
