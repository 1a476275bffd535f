"""Device-side Merlin: the IPA rounds' transcript
steps (append_point L, R; challenge_scalar u; u^-1) run on the GPU
(BPP_IPA_DEVICE_MERLIN=1, k_ipa_transcript_step) with no host round trip
between rounds.  Outputs must be byte-identical to the host-transcript path
and the oracle: IPA (L, R, a, b) and the transcript state after the IPA,
and whole 52-card proofs vs the serial C prover.  Reference: merlin 3.0.0
through transcript_protocol.rs:45-47,62-67."""
import pytest

from oracle import bulletproofs as bp, merlin, ristretto as r255
from oracle.merlin import Rng

pytestmark = pytest.mark.gpu


def sb(x):
    return r255.scalar_bytes(x)


@pytest.fixture(scope="module")
def gens128(ctx):
    import bpperm
    g = bpperm.Gens(ctx, 128)
    yield g
    g.close()


@pytest.mark.parametrize("n", [2, 8, 64, 128])
def test_device_transcript_ipa_matches_oracle(gens128, monkeypatch, n):
    import bpperm
    monkeypatch.setenv("BPP_IPA_DEVICE_MERLIN", "1")
    rng = Rng(700 + n)
    oG, oH = merlin.bulletproof_gens(128)
    Q = rng.point()
    a = [rng.scalar() for _ in range(n)]
    b = [rng.scalar() for _ in range(n)]
    gf = [rng.scalar() for _ in range(n)]
    hf = [rng.scalar() for _ in range(n)]
    ot = merlin.Transcript(b"dev-merlin")
    want = bp.ipa_create(ot, Q, gf, hf, oG[:n], oH[:n], a, b)
    gt = bpperm.Transcript(b"dev-merlin")
    L, R, ga, gb = gens128.ipa_prove(gt, r255.encode(Q), [sb(x) for x in gf], [sb(x) for x in hf],
                                     [sb(x) for x in a], [sb(x) for x in b])
    assert L == want.L and R == want.R
    assert ga == sb(want.a) and gb == sb(want.b)
    # the transcript continues exactly where the host one would
    assert gt.challenge_bytes(b"after", 48) == ot.challenge_bytes(b"after", 48)


def test_device_transcript_proofs_match_host_path(gens128, monkeypatch):
    import bpperm
    from oracle import cport
    pr = bpperm.PermProver(gens128, 52)
    seeds = list(range(3000, 3000 + 70))
    monkeypatch.setenv("BPP_IPA_DEVICE_MERLIN", "0")
    host_p, host_v = pr.prove_batch(seeds)
    monkeypatch.setenv("BPP_IPA_DEVICE_MERLIN", "1")
    dev_p, dev_v = pr.prove_batch(seeds)
    assert dev_p == host_p and dev_v == host_v
    for i in (0, 33, 69):
        want, wv = cport.cpu_prove(52, seeds[i])
        assert dev_p[i] == want and dev_v[i] == b"".join(wv)
    assert pr.verify_batch(dev_p, dev_v)


@pytest.mark.parametrize("k", [52, 5])
def test_device_v_transcript_matches_host_path(gens128, monkeypatch, k):
    """The prover's V phase on the device (BPP_PROVE_DEV_V=1,
    k_prove_v_transcript: 2k V appends + x_perm per lane) gives the same
    proof bytes as the host's 8-way lockstep transcripts (70 proofs: a
    short last wave), also together with the device IPA transcript."""
    import bpperm
    pr = bpperm.PermProver(gens128, k)
    seeds = list(range(4000, 4070))
    monkeypatch.setenv("BPP_PROVE_DEV_V", "0")
    host_p, host_v = pr.prove_batch(seeds)
    monkeypatch.setenv("BPP_PROVE_DEV_V", "1")
    dev_p, dev_v = pr.prove_batch(seeds)
    assert dev_p == host_p and dev_v == host_v
    monkeypatch.setenv("BPP_IPA_DEVICE_MERLIN", "1")
    both_p, _ = pr.prove_batch(seeds)
    assert both_p == host_p
