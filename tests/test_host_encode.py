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


def test_ifma_path_matches_scalar(monkeypatch):
    """The 8-way AVX-512 IFMA batch encoder (host/encode_x8.cpp) against the
    scalar one (BPP_HOST_IFMA=0) on every batch length 1..40 (padded last
    vector, below-8 batches on the scalar path) with identity-torsion lanes
    (W = 0) mixed into the vectors; both against the oracle."""
    import bpperm
    tors = [(0, 1, 1, 0), (0, R.P - 1, 1, 0), (R.SQRT_M1, 0, 1, 0)]
    pts = _rand_points(37, 13)
    pts = pts[:5] + tors[:1] + pts[5:20] + tors[1:] + pts[20:]
    raw = [R.raw_point_bytes(p) for p in pts]
    want = [R.encode(R.ed_double(p)) if i not in (5, 21, 22) else bytes(32) for i, p in enumerate(pts)]
    for n in range(1, len(pts) + 1):
        monkeypatch.setenv("BPP_HOST_IFMA", "1")
        fast = bpperm.double_compress(raw[:n])
        monkeypatch.setenv("BPP_HOST_IFMA", "0")
        slow = bpperm.double_compress(raw[:n])
        assert fast == slow == want[:n], n
