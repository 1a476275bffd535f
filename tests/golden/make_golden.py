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




def config2_inputs(n=1024, seed=1):
    """n = 2^10 Pedersen vector commitment + IPA.
    A = alpha*B_blinding + <a_L, G> + <a_R, H>; transcript "config2" absorbs A,
    y = challenge; IPA on (a_L, a_R) with G_factors = 1, H_factors = y^-i and
    Q = from_uniform_bytes(rng 64 bytes)."""
    from oracle.merlin import bulletproof_gens, pedersen_gens_default
    rng = Rng(seed, b"config2")
    aL = [rng.scalar() for _ in range(n)]
    aR = [rng.scalar() for _ in range(n)]
    alpha = rng.scalar()
    Qraw = rng.bytes(64)
    G, H = bulletproof_gens(n)
    _, Bb = pedersen_gens_default()
    return aL, aR, alpha, Qraw, G, H, Bb


def config2_golden(n=1024, seed=1):
    from oracle import bulletproofs as bp
    from oracle.merlin import Transcript
    aL, aR, alpha, Qraw, G, H, Bb = config2_inputs(n, seed)
    A = r255.encode(bp.msm([alpha] + aL + aR, [Bb] + G + H))
    tr = Transcript(b"config2")
    tr.append_point(b"A", A)
    y = tr.challenge_scalar(b"y")
    yinv = bp.powers(r255.scalar_inv(y), n)
    Q = r255.from_uniform_bytes(Qraw)
    pf = bp.ipa_create(tr, Q, [1] * n, yinv, G, H, aL, aR)
    return {"n": n, "seed": seed, "A": A.hex(), "L": [x.hex() for x in pf.L], "R": [x.hex() for x in pf.R],
            "a": r255.scalar_bytes(pf.a).hex(), "b": r255.scalar_bytes(pf.b).hex()}


def config1_golden(k=52, seed=0):
    """52-card permutation proof (sound mode), seed 0."""
    from oracle import bulletproofs as bp
    pf, perm = bp.ac_prove(k, seed)
    assert bp.ac_verify(k, pf)
    return {"k": k, "seed": seed, "label": "bp-perm", "perm": perm, "V": [v.hex() for v in pf.V],
            "proof": pf.to_bytes().hex()}


def write_protocol():
    import time
    t = time.time()
    c1 = config1_golden()
    t1 = time.time() - t
    c2 = config2_golden()
    out = {"generator": "tests/golden/make_golden.py write_protocol()", "config1": c1, "config2": c2,
           "oracle_seconds": {"config1": t1, "config2": time.time() - t - t1}}
    (HERE / "protocol.json").write_text(json.dumps(out, indent=1))
    print("wrote", HERE / "protocol.json", out["oracle_seconds"])


if __name__ == "__main__":
    which = sys.argv[1:] or ["msm", "protocol"]
    if "msm" in which:
        (HERE / "msm.json").write_text(json.dumps({"generator": "tests/golden/make_golden.py", "cases": msm_cases()}))
        print("wrote", HERE / "msm.json")
    if "protocol" in which:
        write_protocol()
