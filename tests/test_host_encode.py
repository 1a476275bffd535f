"""Host batch encoding of doubled points (bpp_points_double_compress, the
prover's replacement for a per-point inverse square root on small batches)
against the oracle's RFC 9496 encode of 2P.  Host code only: no GPU."""
import os
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

from oracle import ristretto as R  # noqa: E402


def _rand_points(n, seed):
    rng = random.Random(seed)
    pts = []
    for _ in range(n):
        p = R.from_uniform_bytes(bytes(rng.getrandbits(8) for _ in range(64)))
        lam = rng.randrange(1, R.P)  # any projective representative
        pts.append(tuple(c * lam % R.P for c in p))
    return pts


def test_double_compress_matches_oracle():
    import bpperm
    pts = _rand_points(64, 7)
    got = bpperm.double_compress([R.raw_point_bytes(p) for p in pts])
    assert got == [R.encode(R.ed_double(p)) for p in pts]


def test_double_compress_torsion_and_identity():
    import bpperm
    tors = [(0, 1, 1, 0), (0, R.P - 1, 1, 0), (R.SQRT_M1, 0, 1, 0), (R.P - R.SQRT_M1, 0, 1, 0)]
    base = _rand_points(4, 11)
    pts = list(tors) + [R.ed_add(p, t) for p in base for t in tors]
    got = bpperm.double_compress([R.raw_point_bytes(p) for p in pts])
    want = [bytes(32)] * 4 + [R.encode(R.ed_double(p)) for p in base for _ in tors]
    assert got == want


def test_double_compress_empty():
    import bpperm
    assert bpperm.double_compress([]) == []
