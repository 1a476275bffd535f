"""Writes tests/golden/compat_k3_seed0.json: the compat-mode restatement
(oracle/compat.py, the reference's test_first as written) at k = 3 (the
reference's test_1: test_first(6, 7)), seed 0 -- a regression pin of the
restatement (parity unpinned: the reference's randomness is thread_rng).
    python tests/golden/make_compat_golden.py"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import compat, ristretto as r255  # noqa: E402


def summary(run):
    e = r255.encode
    sc = r255.scalar_bytes
    return {
        "k": run.k,
        "A_I": e(run.A_I).hex(), "A_O": e(run.A_O).hex(), "S": e(run.S).hex(),
        "V": [e(p).hex() for p in run.V],
        "y": sc(run.y).hex(), "z": sc(run.z).hex(), "x": sc(run.x).hex(),
        "T": [e(p).hex() for p in run.T],
        "tau_x": sc(run.tau_x).hex(), "mu": sc(run.mu).hex(), "t": sc(run.t).hex(),
        "l": [sc(v).hex() for v in run.l], "r": [sc(v).hex() for v in run.r],
        "verify": run.verify["result"],
    }


if __name__ == "__main__":
    out = ROOT / "tests" / "golden" / "compat_k3_seed0.json"
    out.write_text(json.dumps(summary(compat.compat_prove(3, 0)), indent=1) + "\n")
    print(out)
