"""The reference's own prover flow, AS WRITTEN (compat mode: test_first,
lib.rs:160-233, with its defects), driven through the drop-in boundary:
every group operation at the reference's call sites -- the V commitments
(PedersenGens::commit, weights.rs:60), A_I / A_O / S
(vartime_multiscalar_mul, circuit_lib.rs:187-229), the T_i (:363-412), and
the verifier's MSMs (h_ = H y^-i, weights_L/R/O, the t-check candidates, P,
cand_P; :491-575) -- and the Merlin transcript run in libbpperm.so
(bpp_pedersen_commit_batch, bpp_vec_commit, bpp_msm, bpp_transcript_*),
and must equal the oracle's restatement (oracle/compat.py) element for
element, including where the reference's verify fails."""
import pytest

from oracle import compat
from oracle import ristretto as r255

pytestmark = pytest.mark.gpu
L = r255.L


class AbiEngine(compat.Engine):
    """compat.Engine over the C ABI: points cross as compressed bytes."""

    def __init__(self, ctx):
        super().__init__()
        self.ctx = ctx
        self.gens = None
        self.calls = {"msm": 0, "commit": 0, "vec_commit": 0}

    def set_gens(self, B, Bb, G, H):
        import bpperm
        super().set_gens(B, Bb, G, H)
        enc = r255.encode
        self.gens = bpperm.Gens(self.ctx, points=([enc(p) for p in G], [enc(p) for p in H], enc(B), enc(Bb)))

    def msm(self, scalars, points):
        self.calls["msm"] += 1
        out = self.ctx.msm([r255.scalar_bytes(s % L) for s in scalars], [r255.encode(p) for p in points])
        return r255.decode(out)

    def commit(self, v, blind):
        self.calls["commit"] += 1
        return r255.decode(self.gens.pedersen_commit([r255.scalar_bytes(v)], [r255.scalar_bytes(blind)])[0])

    def vec_commit(self, blind, a, b=None):
        self.calls["vec_commit"] += 1
        sb = r255.scalar_bytes
        out = self.gens.vec_commit(sb(blind), [sb(x) for x in a], [sb(x) for x in b] if b is not None else None)
        return r255.decode(out)

    def transcript(self, label):
        import bpperm

        class Tr:  # bpperm.Transcript with the oracle's int challenges
            def __init__(self):
                self.t = bpperm.Transcript(label)

            def arithmetic_domain_sep(self, n):
                self.t.arithmetic_domain_sep(n)

            def append_message(self, lab, msg):
                self.t.append_message(lab, msg)

            def challenge_scalar(self, lab):
                return int.from_bytes(self.t.challenge_scalar(lab), "little")

        return Tr()


@pytest.mark.parametrize("k", [3, 52])
def test_reference_flow_through_the_abi(ctx, k):
    ref = compat.compat_prove(k, 0)
    eng = AbiEngine(ctx)
    got = compat.compat_prove(k, 0, engine=eng)
    enc = r255.encode
    # every commitment the prover sends, and the challenges they bind
    assert [enc(p) for p in got.V] == [enc(p) for p in ref.V]
    for name in ("A_I", "A_O", "S"):
        assert enc(getattr(got, name)) == enc(getattr(ref, name)), name
    assert [enc(p) for p in got.T] == [enc(p) for p in ref.T]
    assert (got.y, got.z, got.x) == (ref.y, ref.z, ref.x)
    assert (got.tau_x, got.mu, got.t, got.l, got.r) == (ref.tau_x, ref.mu, ref.t, ref.l, ref.r)
    # the verifier's group elements, and its outcome: Err at the t-check
    for key in ("weights_L", "weights_R", "weights_O", "gt_htau_cand", "gt_htau", "P", "cand_P"):
        assert enc(got.verify[key]) == enc(ref.verify[key]), key
    assert [enc(p) for p in got.verify["h_"]] == [enc(p) for p in ref.verify["h_"]]
    assert got.verify["result"] == ref.verify["result"] == "Err(tau)"
    n, m = 2 * k, 2 * k + 1
    assert eng.calls == {"commit": m + 5, "vec_commit": 3, "msm": n + 7}
    eng.gens.close()
