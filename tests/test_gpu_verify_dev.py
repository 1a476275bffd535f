"""GPU batch verification with the Fiat-Shamir replay on the device
(bpp_perm_verify_begin_dev / bpp_perm_verify_batch: k_verify_replay_g, one
16-lane group per proof; k_verify_consts makes each proof's weight from the
batch's verifier seed and its own r; no inverses, no host round trip;
reference verify, circuit_lib.rs:478-585; transcript_protocol.rs:48-67).

Parity: every proof's r challenge from the device replay is byte-equal to the
host replay (host/merlin.h, itself KAT-pinned against merlin 3.0.0), and a
device job's partial MSM sums are byte-equal to a host job's on the same
window ranges (identical records -> identical scalars -> the same partial
point per window range).  Covered: accept; rejection of a tampered scalar, a swapped V, a
non-canonical scalar, an identity point and an undecodable point; the
8-range window split and a 4-slice proof split; config 5 at its full size
(4096 proofs, one 520,450-term MSM)."""
import pytest

pytestmark = pytest.mark.gpu

K = 52
PLEN = 8 * 32 + 3 * 32 + 14 * 32 + 2 * 32  # bpp_perm_proof_len(52)


@pytest.fixture(scope="module")
def setup(ctx):
    import bpperm
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, K)
    proofs, Vs = pr.prove_batch(list(range(7000, 7000 + 96)))
    yield g, pr, proofs, Vs
    g.close()


SEED = bytes(range(32))  # (a fixed verifier seed: tests compare partials across jobs)


def _window_partials(pr, job, ranks, seed=SEED):
    from bpperm.dist import window_ranges
    c, W = job.windows()
    return [pr.verify_partial(job, seed, 0, wb, we) for wb, we in window_ranges(W, ranks)]


def test_device_r_equals_host_r(setup, ctx):
    import bpperm
    _, pr, proofs, Vs = setup
    hj = bpperm.VerifyJob(K, proofs, Vs)
    dj = bpperm.VerifyJob(K, proofs, Vs, ctx=ctx)
    assert hj.ok and dj.ok
    assert dj.r == hj.r and len(dj.r) == 32 * len(proofs)
    assert dj.terms() == hj.terms()
    # the same records on both paths: the same group element per window range
    # (compared encoded: a raw partial's projective representation depends
    # on the order of the bucket additions)
    hp = _window_partials(pr, hj, 8)
    dp = _window_partials(pr, dj, 8)
    assert [bpperm.partials_finish([p]) for p in hp] == [bpperm.partials_finish([p]) for p in dp]
    assert bpperm.partials_is_identity(dp)
    hj.close()
    dj.close()


def test_device_job_other_label(setup, ctx):
    """The transcript label reaches the device replay (shared prefix state)."""
    import bpperm
    gens, _, _, _ = setup
    pr = bpperm.PermProver(gens, K, label=b"another label, longer than the rate's first block? no")
    proofs, Vs = pr.prove_batch([1, 2, 3, 4, 5])
    hj = bpperm.VerifyJob(K, proofs, Vs, label=pr.label)
    dj = bpperm.VerifyJob(K, proofs, Vs, label=pr.label, ctx=ctx)
    assert dj.r == hj.r
    assert pr.verify_batch(proofs, Vs)
    # the wrong label: every challenge differs and the batch rejects
    assert not bpperm.PermProver(gens, K).verify_batch(proofs, Vs)
    hj.close()
    dj.close()


def test_small_circuits(ctx):
    """Other circuit sizes (lg = 2..5) through the device replay."""
    import bpperm
    g = bpperm.Gens(ctx, 64)
    for k in (2, 3, 7, 16):
        pr = bpperm.PermProver(g, k)
        proofs, Vs = pr.prove_batch(list(range(40 + k, 52 + k)))
        hj = bpperm.VerifyJob(k, proofs, Vs)
        dj = bpperm.VerifyJob(k, proofs, Vs, ctx=ctx)
        assert dj.r == hj.r, k
        assert pr.verify_batch(proofs, Vs), k
        assert pr.verify(proofs[3], Vs[3]), k
        hj.close()
        dj.close()
    g.close()


def _tampered(proofs, i, off, xor):
    bad = list(proofs)
    b = bytearray(bad[i])
    b[off] ^= xor
    bad[i] = bytes(b)
    return bad


def test_device_rejects(setup, ctx):
    import bpperm
    _, pr, proofs, Vs = setup
    assert pr.verify_batch(proofs, Vs)
    # t_hat, stays canonical (low byte)
    assert not pr.verify_batch(_tampered(proofs, 37, 8 * 32 + 70, 1), Vs)
    # a V commitment swapped between proofs
    bv = list(Vs)
    bv[3], bv[4] = bv[4], bv[3]
    assert not pr.verify_batch(proofs, bv)
    # a non-canonical scalar (tau_x top byte): rejected by the replay itself
    nc = _tampered(proofs, 11, 8 * 32 + 31, 0xF0)
    assert bpperm.VerifyJob(K, nc, Vs, ctx=ctx).ok is False
    assert not pr.verify_batch(nc, Vs)
    # the identity encoding for A_O (validate_and_append_point)
    zp = list(proofs)
    b = bytearray(zp[50])
    b[32:64] = bytes(32)
    zp[50] = bytes(b)
    assert bpperm.VerifyJob(K, zp, Vs, ctx=ctx).ok is False
    assert bpperm.VerifyJob(K, zp, Vs).ok is False
    # an undecodable L_0 (high bit set: not a canonical field encoding)
    ud = _tampered(proofs, 60, 11 * 32 + 31, 0x80)
    assert not pr.verify_batch(ud, Vs)
    assert not pr.verify(ud[60], Vs[60])
    uj = bpperm.VerifyJob(K, ud, Vs, ctx=ctx)
    assert uj.ok  # (the replay absorbs the bytes; the decompression beside it rejects)
    assert pr.verify_partial(uj, SEED, 0, 0, uj.windows()[1]) is None
    uj.close()
    # the untampered batch still verifies on the same context afterwards
    assert pr.verify_batch(proofs, Vs)


def test_device_proof_split(setup, ctx):
    """4 proof slices, one context per "rank" (a device job lives in its
    context's workspaces): same group element as the window split."""
    import bpperm
    from bpperm.dist import point_ranges
    gens, pr, proofs, Vs = setup
    bad = _tampered(proofs, 5, 8 * 32 + 33, 2)  # mu: a non-identity sum
    ctxs = [bpperm.Context(0) for _ in range(4)]
    try:
        jobs = [(b, bpperm.VerifyJob(K, bad[b:e], Vs[b:e], ctx=c))
                for (b, e), c in zip(point_ranges(len(bad), 4), ctxs)]
        r_all = b"".join(j.r for _, j in jobs)
        prs = [bpperm.PermProver(gens, K, ctx=c) for c in ctxs]
        parts = [p.verify_partial(j, SEED, b, 0, j.windows()[1]) for p, (b, j) in zip(prs, jobs)]
        whole = bpperm.VerifyJob(K, bad, Vs, ctx=ctx)
        assert whole.r == r_all
        wparts = _window_partials(pr, whole, 8)
        assert bpperm.partials_finish(parts) == bpperm.partials_finish(wparts) != bytes(32)
        whole.close()
        for _, j in jobs:
            j.close()
    finally:
        for c in ctxs:
            c.close()


def test_superseded_device_job_is_refused(setup, ctx):
    import bpperm
    from bpperm._lib import BppError
    _, pr, proofs, Vs = setup
    j1 = bpperm.VerifyJob(K, proofs[:8], Vs[:8], ctx=ctx)
    j2 = bpperm.VerifyJob(K, proofs[8:16], Vs[8:16], ctx=ctx)
    with pytest.raises(BppError):
        pr.verify_partial(j1, SEED, 0, 0, j1.windows()[1])
    assert bpperm.partials_is_identity([pr.verify_partial(j2, SEED, 0, 0, j2.windows()[1])])
    j1.close()
    j2.close()


def test_config5_full_size(ctx):
    """Config 5 at full size: 4096 proofs in one verification (one 520,450-
    term MSM).  r challenges byte-equal to the host replay; accept; the
    8-range window split adds up to the identity; one tampered proof is
    rejected by the batch and by the split."""
    import bpperm
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, K)
    proofs, Vs = [], []
    for b in range(0, 4096, 256):
        p, v = pr.prove_batch(list(range(900_000 + b, 900_000 + b + 256)))
        proofs += p
        Vs += v
    hj = bpperm.VerifyJob(K, proofs, Vs)
    dj = bpperm.VerifyJob(K, proofs, Vs, ctx=ctx)
    assert dj.r == hj.r
    assert dj.terms() == 258 + 4096 * 127 == 520_450
    hj.close()
    parts = _window_partials(pr, dj, 8)
    assert bpperm.partials_is_identity(parts)
    assert not bpperm.partials_is_identity(parts[:7])
    dj.close()
    assert pr.verify_batch(proofs, Vs)
    bad = _tampered(proofs, 2049, 8 * 32 + 70, 1)
    assert not pr.verify_batch(bad, Vs)
    bj = bpperm.VerifyJob(K, bad, Vs, ctx=ctx)
    assert bj.ok  # (well-formed: only the MSM check fails)
    assert not bpperm.partials_is_identity(_window_partials(pr, bj, 8))
    bj.close()
    # the proof points are decompressed per upload chunk (4 chunks here, 3
    # uneven ones of 333 / 333 / 334 proofs at 1000): an undecodable point
    # in the last chunk, in a middle one, and in both is still caught
    for n in (4096, 1000):
        assert pr.verify_batch(proofs[:n], Vs[:n])
        for where in ([n - 1], [n // 2], [n // 3, n - 2]):
            ud = list(proofs[:n])
            for i in where:
                ud = _tampered(ud, i, 11 * 32 + 31, 0x80)  # L_0's top bit
            assert not pr.verify_batch(ud, Vs[:n]), (n, where)
    g.close()


def test_prover_scratch_keyed_on_generators(ctx):
    """one thread proves the same (P, k) against generator
    sets of different sizes; the cached A_I/A_O/S term indices embed G->n, so
    both batches must verify."""
    import bpperm
    g1 = bpperm.Gens(ctx, 128)
    g2 = bpperm.Gens(ctx, 256)
    for g in (g1, g2, g1):
        pr = bpperm.PermProver(g, 52)
        proofs, Vs = pr.prove_batch(list(range(60, 68)))
        assert pr.verify_batch(proofs, Vs)
    g1.close()
    g2.close()


def test_weights_follow_the_seed(setup, ctx):
    """The batch weights come from the verifier's seed (and each proof's own
    r): an honest batch verifies under any seed, a tampered one under none
    of several, and two seeds give different partials for the same window
    range (the weights are not fixed by the proofs)."""
    import bpperm
    _, pr, proofs, Vs = setup
    dj = bpperm.VerifyJob(K, proofs, Vs, ctx=ctx)
    s1, s2 = bpperm.verify_seed(), bpperm.verify_seed()
    assert s1 != s2
    p1, p2 = _window_partials(pr, dj, 2, s1), _window_partials(pr, dj, 2, s2)
    assert bpperm.partials_is_identity(p1) and bpperm.partials_is_identity(p2)
    assert bpperm.partials_finish(p1[:1]) != bpperm.partials_finish(p2[:1])
    dj.close()
    bad = _tampered(proofs, 9, 8 * 32 + 70, 1)
    bj = bpperm.VerifyJob(K, bad, Vs, ctx=ctx)
    for _ in range(3):
        assert not bpperm.partials_is_identity(_window_partials(pr, bj, 2, bpperm.verify_seed()))
    bj.close()
