"""GPU parity for the protocol rows: generators, Pedersen commitments,
vector commitments, Merlin transcript, inner-product argument."""
import pytest

from oracle import bulletproofs as bp, merlin, ristretto as r255
from oracle.merlin import Rng

pytestmark = pytest.mark.gpu


def sb(s):
    return r255.scalar_bytes(s)


@pytest.fixture(scope="module")
def gens16(ctx):
    import bpperm
    g = bpperm.Gens(ctx, 16)
    yield g
    g.close()


def test_gens_match_bulletproofs_spec(gens16):
    G, H, B, Bb = gens16.export()
    oG, oH = merlin.bulletproof_gens(16)
    ob, obb = merlin.pedersen_gens_default()
    assert G == [r255.encode(p) for p in oG]
    assert H == [r255.encode(p) for p in oH]
    assert B == r255.encode(ob) and Bb == r255.encode(obb)


def test_pedersen_commit_batch(gens16):
    rng = Rng(5)
    L = r255.L
    v = [rng.scalar() for _ in range(50)] + [0, 1, L - 1, 2**252, 0]
    g = [rng.scalar() for _ in range(50)] + [L - 1, 0, 7, 2**252 - 1, 0]
    got = gens16.pedersen_commit([sb(x) for x in v], [sb(x) for x in g])
    B, Bb = merlin.pedersen_gens_default()
    want = [r255.encode(r255.msm([a, c], [B, Bb])) for a, c in zip(v, g)]
    assert got == want
    assert got[-1] == bytes(32)  # the identity (its double-encoding W is zero)


def test_pedersen_commit_batch_large(gens16):
    """2 100 commitments (the 8-group kernel, 263 lanes of the batched double
    encoding, 4 points in the last): 37 distinct pairs, identity included,
    repeated in a scrambled order, each checked against the oracle."""
    rng = Rng(55)
    L = r255.L
    pairs = [(rng.scalar(), rng.scalar()) for _ in range(33)] + [(0, 0), (3, 0), (0, L - 1), (L - 1, L - 1)]
    order = [(i * 17 + i // 37) % len(pairs) for i in range(2100)]
    got = gens16.pedersen_commit([sb(pairs[j][0]) for j in order], [sb(pairs[j][1]) for j in order])
    B, Bb = merlin.pedersen_gens_default()
    want = [r255.encode(r255.msm([a, c], [B, Bb])) for a, c in pairs]
    assert got == [want[j] for j in order]


def test_vec_commit(gens16):
    rng = Rng(6)
    oG, oH = merlin.bulletproof_gens(16)
    _, Bb = merlin.pedersen_gens_default()
    a = [rng.scalar() for _ in range(16)]
    b = [rng.scalar() for _ in range(16)]
    blind = rng.scalar()
    assert gens16.vec_commit(sb(blind), [sb(x) for x in a], [sb(x) for x in b]) == \
        r255.encode(bp.msm([blind] + a + b, [Bb] + oG + oH))
    assert gens16.vec_commit(sb(blind), [sb(x) for x in a[:9]]) == \
        r255.encode(bp.msm([blind] + a[:9], [Bb] + oG[:9]))


def test_transcript_matches_merlin_kat():
    import bpperm
    t = bpperm.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == \
        "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"
    o = merlin.Transcript(b"x")
    t = bpperm.Transcript(b"x")
    for i in range(5):
        o.append_u64(b"n", i)
        t.append_u64(b"n", i)
        o.append_message(b"m" * i, bytes(range(i * 40)))
        t.append_message(b"m" * i, bytes(range(i * 40)))
        assert t.challenge_scalar(b"c") == sb(o.challenge_scalar(b"c"))


@pytest.mark.parametrize("n", [1, 2, 8, 16])
def test_ipa_prove_matches_oracle_and_verifies(ctx, gens16, n):
    import bpperm
    rng = Rng(100 + n)
    oG, oH = merlin.bulletproof_gens(16)
    G, H = oG[:n], oH[:n]
    Q = rng.point()
    a = [rng.scalar() for _ in range(n)]
    b = [rng.scalar() for _ in range(n)]
    gf = [rng.scalar() for _ in range(n)]
    hf = [rng.scalar() for _ in range(n)]
    want = bp.ipa_create(merlin.Transcript(b"ipa-test"), Q, gf, hf, G, H, a, b)
    L, R, ga, gb = gens16.ipa_prove(bpperm.Transcript(b"ipa-test"), r255.encode(Q), [sb(x) for x in gf],
                                    [sb(x) for x in hf], [sb(x) for x in a], [sb(x) for x in b])
    assert L == want.L and R == want.R
    assert ga == sb(want.a) and gb == sb(want.b)
    P = bp.msm([x * f for x, f in zip(a, gf)] + [x * f for x, f in zip(b, hf)] + [bp.inner(a, b)], G + H + [Q])
    args = (n, [sb(x) for x in gf], [sb(x) for x in hf], r255.encode(P), r255.encode(Q), L, R, ga, gb)
    assert gens16.ipa_verify(bpperm.Transcript(b"ipa-test"), *args)
    if n > 1:  # with no rounds the transcript never reaches a challenge
        assert not gens16.ipa_verify(bpperm.Transcript(b"other"), *args)
    bad = list(args)
    bad[7] = sb((want.a + 1) % r255.L)
    assert not gens16.ipa_verify(bpperm.Transcript(b"ipa-test"), *bad)


@pytest.mark.parametrize("mode", ["var", "fb", "dt"])
def test_ipa_and_vec_commit_both_msm_engines(ctx, gens16, monkeypatch, mode):
    import bpperm
    # var: per-window Pippenger; fb: window tables + shared buckets;
    # dt: direct radix-2^8 tables (default for small MSMs over generators)
    monkeypatch.setenv("BPP_MSM_DT", "1" if mode == "dt" else "0")
    monkeypatch.setenv("BPP_MSM_FB", "1" if mode == "fb" else "0")
    rng = Rng(300)
    oG, oH = merlin.bulletproof_gens(16)
    _, Bb = merlin.pedersen_gens_default()
    n = 16
    Q = rng.point()
    a = [rng.scalar() for _ in range(n)]
    b = [rng.scalar() for _ in range(n)]
    blind = rng.scalar()
    assert gens16.vec_commit(sb(blind), [sb(x) for x in a], [sb(x) for x in b]) == \
        r255.encode(bp.msm([blind] + a + b, [Bb] + oG + oH))
    ones = [1] * n
    want = bp.ipa_create(merlin.Transcript(b"ipa-fb"), Q, ones, ones, oG, oH, a, b)
    L, R, ga, gb = gens16.ipa_prove(bpperm.Transcript(b"ipa-fb"), r255.encode(Q), None, None,
                                    [sb(x) for x in a], [sb(x) for x in b])
    assert L == want.L and R == want.R and ga == sb(want.a) and gb == sb(want.b)
    P = bp.msm(a + b + [bp.inner(a, b)], oG + oH + [Q])
    assert gens16.ipa_verify(bpperm.Transcript(b"ipa-fb"), n, None, None, r255.encode(P), r255.encode(Q),
                             L, R, ga, gb)


def test_ipa_q_slot_shared_gens_two_contexts(ctx, gens16):
    """bpp_ipa_prove writes Q into the generators' spare slot for the call
    (gens.h qslot, under a per-set mutex): two contexts proving with
    different Q on one generator set from two threads get their own proofs,
    and an undecodable Q is refused (BPP_ERR_DECOMPRESS)."""
    import ctypes as C
    import threading

    import bpperm
    rng = Rng(900)
    oG, oH = merlin.bulletproof_gens(16)
    n = 16
    cases = []
    for i in range(4):
        Q = rng.point()
        a = [rng.scalar() for _ in range(n)]
        b = [rng.scalar() for _ in range(n)]
        want = bp.ipa_create(merlin.Transcript(b"qslot"), Q, [1] * n, [1] * n, oG, oH, a, b)
        cases.append((r255.encode(Q), b"".join(sb(x) for x in a), b"".join(sb(x) for x in b), want))
    ctx2 = bpperm.Context(0)
    lib = ctx.lib
    errs = []

    def run(c, idx):
        try:
            for _ in range(3):
                for i in idx:
                    Qe, ab, bb, want = cases[i]
                    tr = bpperm.Transcript(b"qslot")
                    Lo, Ro = C.create_string_buffer(32 * 4), C.create_string_buffer(32 * 4)
                    ao, bo = C.create_string_buffer(32), C.create_string_buffer(32)
                    rc = lib.bpp_ipa_prove(c.h, gens16.h, tr.h, C.c_char_p(Qe), None, None, C.c_char_p(ab),
                                           C.c_char_p(bb), n, Lo, Ro, ao, bo)
                    tr.close()
                    L = [Lo.raw[32 * k: 32 * k + 32] for k in range(4)]
                    R = [Ro.raw[32 * k: 32 * k + 32] for k in range(4)]
                    if rc != 0 or L != want.L or R != want.R or ao.raw != sb(want.a) or bo.raw != sb(want.b):
                        errs.append((i, rc))
        except Exception as e:  # (reported below)
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(ctx, [0, 1])), threading.Thread(target=run, args=(ctx2, [2, 3]))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ctx2.close()
    assert errs == []
    bad = bytes([1]) + bytes(31)  # a nonzero encoding that is not a ristretto point (odd)
    with pytest.raises(bpperm.BppError):
        gens16.ipa_prove(bpperm.Transcript(b"qslot"), bad, None, None, cases[0][1], cases[0][2])
