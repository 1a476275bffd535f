"""Golden protocol vectors (tests/golden/protocol.json, made by
tests/golden/make_golden.py from the oracle).

CPU: the oracle reproduces config 1 (52-card sound-mode proof, seed 0) and
verifies it.  GPU: the HIP path reproduces config 1 byte-for-byte and config 2
(2^10 vector commitment + IPA) point-for-point."""
import json
from pathlib import Path

import pytest

from oracle import bulletproofs as bp, ristretto as r255

GOLD = json.loads((Path(__file__).parent / "golden" / "protocol.json").read_text())


def test_oracle_reproduces_config1():
    c1 = GOLD["config1"]
    pf, perm = bp.ac_prove(c1["k"], c1["seed"])
    assert perm == c1["perm"]
    assert pf.to_bytes().hex() == c1["proof"]
    assert [v.hex() for v in pf.V] == c1["V"]


def test_config1_fixture_shape():
    c1 = GOLD["config1"]
    k = c1["k"]
    assert len(c1["V"]) == 2 * k + 1
    assert sorted(c1["perm"]) == list(range(k))
    assert len(bytes.fromhex(c1["proof"])) == 32 * (8 + 3 + 2 * 7 + 2)


@pytest.mark.gpu
def test_gpu_config1_bit_exact(ctx):
    import bpperm
    c1 = GOLD["config1"]
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, c1["k"], label=c1["label"].encode())
    proof, V, perm = pr.prove(c1["seed"])
    assert perm == c1["perm"]
    assert [v.hex() for v in V] == c1["V"]
    assert proof.hex() == c1["proof"]
    assert pr.verify(proof, V)
    g.close()


@pytest.mark.gpu
def test_gpu_config2_commit_ipa(ctx):
    import bpperm
    import sys
    sys.path.insert(0, str(Path(__file__).parent / "golden"))
    from make_golden import config2_inputs
    c2 = GOLD["config2"]
    n = c2["n"]
    aL, aR, alpha, Qraw, _, _, _ = config2_inputs(n, c2["seed"])
    g = bpperm.Gens(ctx, n)
    sb = r255.scalar_bytes
    A = g.vec_commit(sb(alpha), [sb(x) for x in aL], [sb(x) for x in aR])
    assert A.hex() == c2["A"]
    tr = bpperm.Transcript(b"config2")
    tr.append_point(b"A", A)
    y = int.from_bytes(tr.challenge_scalar(b"y"), "little")
    yinv = bp.powers(r255.scalar_inv(y), n)
    Q = r255.encode(r255.from_uniform_bytes(Qraw))
    L, R, a, b = g.ipa_prove(tr, Q, None, [sb(x) for x in yinv], [sb(x) for x in aL], [sb(x) for x in aR])
    assert [x.hex() for x in L] == c2["L"] and [x.hex() for x in R] == c2["R"]
    assert a.hex() == c2["a"] and b.hex() == c2["b"]
    g.close()
