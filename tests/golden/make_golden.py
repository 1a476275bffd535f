"""Generate the committed golden vectors under tests/golden/ from the CPU
oracle (oracle/, pinned by tests/test_oracle_kat.py).

    python tests/golden/make_golden.py

msm.json: MSM cases at the sizes SURVEY.md §7 lists (1, 2, 3, 64, 190, 1024):
inputs are seeded uniform bytes (points = from_uniform_bytes) and seeded wide
scalars; the expected output is the compressed sum.  Sizes 189/190 straddle
dalek's Straus/Pippenger switch.
"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

from oracle import ristretto as r255  # noqa: E402
from oracle.merlin import Rng  # noqa: E402


def msm_cases():
    cases = []
    for n, seed in [(1, 1), (2, 2), (3, 3), (64, 64), (189, 189), (190, 190), (1024, 1024)]:
        rng = Rng(seed, b"golden-msm")
        raw = [rng.bytes(64) for _ in range(n)]
        sc = [rng.scalar() for _ in range(n)]
        pts = [r255.from_uniform_bytes(b) for b in raw]
        want = r255.msm_pippenger(sc, pts, 6 if n < 500 else 8)
        cases.append({
            "n": n, "seed": seed,
            "uniform": "".join(b.hex() for b in raw),
            "points": "".join(r255.encode(p).hex() for p in pts),
            "scalars": "".join(r255.scalar_bytes(s).hex() for s in sc),
            "result": r255.encode(want).hex(),
        })
    # edge scalars (0, 1, l-1, 2^252, ...) on 8 points
    rng = Rng(7, b"golden-msm-edge")
    raw = [rng.bytes(64) for _ in range(8)]
    pts = [r255.from_uniform_bytes(b) for b in raw]
    L = r255.L
    sc = [0, 1, L - 1, 2**252, 2**128 + 7, L - 2, 12345, 2**252 - 1]
    cases.append({"n": 8, "seed": "edge", "uniform": "".join(b.hex() for b in raw),
                  "points": "".join(r255.encode(p).hex() for p in pts),
                  "scalars": "".join(r255.scalar_bytes(s).hex() for s in sc),
                  "result": r255.encode(r255.msm(sc, pts)).hex()})
    return cases


if __name__ == "__main__":
    (HERE / "msm.json").write_text(json.dumps({"generator": "tests/golden/make_golden.py", "cases": msm_cases()}))
    print("wrote", HERE / "msm.json")
