"""GPU parity: point codec and Ristretto MSM through the C ABI vs the oracle.

Bit-exact comparison of canonical 32-byte encodings (SURVEY.md §7 'hard
parts': only canonical encodings are compared)."""
import pytest

from oracle import ristretto as r255
from oracle.merlin import Rng

pytestmark = pytest.mark.gpu


def _points(seed, n):
    rng = Rng(seed, b"test-points")
    raw = [rng.bytes(64) for _ in range(n)]
    return raw, [r255.from_uniform_bytes(b) for b in raw]


def _scalars(seed, n):
    rng = Rng(seed, b"test-scalars")
    return [rng.scalar() for _ in range(n)]


def test_from_uniform_and_compress(ctx):
    raw, pts = _points(1, 97)
    tbl = ctx.from_uniform(raw)
    got = tbl.compress()
    assert got == [r255.encode(p) for p in pts]


def test_decompress_roundtrip(ctx):
    _, pts = _points(2, 65)
    enc = [r255.encode(p) for p in pts] + [r255.encode(r255.IDENTITY), r255.encode(r255.BASEPOINT)]
    tbl = ctx.decompress(enc)
    assert tbl.compress() == enc


def test_decompress_rejects_invalid(ctx):
    import bpperm
    bad = bytearray(r255.encode(r255.BASEPOINT))
    bad[0] ^= 1  # negative s
    with pytest.raises(bpperm.BppError) as ei:
        ctx.decompress([r255.encode(r255.BASEPOINT), bytes(bad)])
    assert ei.value.name == "BPP_ERR_DECOMPRESS"


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 190, 300])
def test_msm_matches_oracle(ctx, n):
    raw, pts = _points(10 + n, n)
    sc = _scalars(20 + n, n)
    enc = [r255.encode(p) for p in pts]
    got = ctx.msm([r255.scalar_bytes(s) for s in sc], enc)
    want = r255.encode(r255.msm_pippenger(sc, pts, 6))
    assert got == want


def test_msm_edge_scalars(ctx):
    raw, pts = _points(5, 8)
    L = r255.L
    sc = [0, 1, L - 1, 2**252, 2**128 + 7, (1 << 253) - 1 - ((1 << 253) - L), 12345, L - 2]
    sc = [s % L for s in sc]
    got = ctx.msm([r255.scalar_bytes(s) for s in sc], [r255.encode(p) for p in pts])
    assert got == r255.encode(r255.msm(sc, pts))


def test_msm_rejects_noncanonical(ctx):
    import bpperm
    _, pts = _points(6, 2)
    with pytest.raises(bpperm.BppError) as ei:
        ctx.msm([r255.L.to_bytes(32, "little"), r255.scalar_bytes(1)], [r255.encode(p) for p in pts])
    assert ei.value.name == "BPP_ERR_NONCANONICAL"


def test_msm_batch(ctx):
    raw, pts = _points(7, 40)
    tbl = ctx.from_uniform(raw)
    sizes = [1, 5, 40, 0, 13, 2]
    offs = [0]
    idx = []
    scal = []
    rng = Rng(99)
    for k, m in enumerate(sizes):
        for j in range(m):
            idx.append((7 * j + k) % 40)
            scal.append(rng.scalar())
        offs.append(len(idx))
    got = ctx.msm_batch(offs, [r255.scalar_bytes(s) for s in scal], idx, tbl)
    for k in range(len(sizes)):
        a, b = offs[k], offs[k + 1]
        want = r255.encode(r255.msm_pippenger(scal[a:b], [pts[i] for i in idx[a:b]], 5))
        assert got[k] == want, k


def test_msm_window_partials(ctx):
    import bpperm
    n = 300
    raw, pts = _points(8, n)
    tbl = ctx.from_uniform(raw)
    sc = _scalars(9, n)
    sb = b"".join(r255.scalar_bytes(s) for s in sc)
    d = ctx.dev_alloc(len(sb))
    ctx.htod(d, sb)
    c, W = bpperm.msm_windows(n)
    full = ctx.msm_table_dev(d, tbl, n)
    cuts = [0, W // 3, W // 2, W]
    parts = [ctx.msm_table_dev_partial(d, tbl, n, cuts[i], cuts[i + 1]) for i in range(3)]
    assert bpperm.partials_finish(parts) == full
    assert full == r255.encode(r255.msm_pippenger(sc, pts, 6))
    ctx.dev_free(d)


def test_msm_golden_vectors(ctx):
    import json
    from pathlib import Path
    cases = json.loads((Path(__file__).parent / "golden" / "msm.json").read_text())["cases"]
    for case in cases:
        pts = bytes.fromhex(case["points"])
        tbl = ctx.from_uniform(bytes.fromhex(case["uniform"]))
        assert b"".join(tbl.compress()) == pts
        assert ctx.msm(bytes.fromhex(case["scalars"]), pts).hex() == case["result"], case["n"]
        assert ctx.msm_table(bytes.fromhex(case["scalars"]), tbl).hex() == case["result"], case["n"]


def _gpu_decodes(ctx, enc: bytes):
    import bpperm
    try:
        t = ctx.decompress([enc])
    except bpperm.BppError as e:
        assert e.name == "BPP_ERR_DECOMPRESS"
        return None
    out = t.compress()[0]
    t.close()
    return out


def test_rfc9496_bad_encodings_rejected_by_gpu_decoder(ctx):
    """RFC 9496 §A.2 bad encodings (tests/test_oracle_kat.py) through the GPU
    decoder: every one is BPP_ERR_DECOMPRESS, alone and inside a batch of
    valid encodings (bad_index reported)."""
    from test_oracle_kat import BAD_ENCODINGS
    good = [r255.encode(p) for p in _points(5, 9)[1]]
    import bpperm
    for h in BAD_ENCODINGS:
        enc = bytes.fromhex(h)
        with pytest.raises(r255.DecodeError):
            r255.decode(enc)
        assert _gpu_decodes(ctx, enc) is None, h
        with pytest.raises(bpperm.BppError) as ei:
            ctx.decompress(good[:4] + [enc] + good[4:])
        assert ei.value.name == "BPP_ERR_DECOMPRESS"


def test_random_encodings_accept_reject_matches_oracle(ctx):
    """Random 32-byte strings (most invalid: non-canonical, negative or
    non-square) and their low-bit-cleared variants: the GPU decoder accepts
    exactly what the oracle accepts, and re-encodes accepted ones canonically."""
    rng = Rng(77, b"codec-sweep")
    cases = []
    for _ in range(48):
        b = bytearray(rng.bytes(32))
        b[31] &= 0x7F
        cases.append(bytes(b))
        b[0] &= 0xFE  # even s: about half of these are valid encodings
        cases.append(bytes(b))
    agree = accepted = 0
    for enc in cases:
        try:
            want = r255.encode(r255.decode(enc))
        except r255.DecodeError:
            want = None
        got = _gpu_decodes(ctx, enc)
        assert got == want, enc.hex()
        agree += 1
        accepted += want is not None
    assert agree == len(cases) and 0 < accepted < len(cases)
