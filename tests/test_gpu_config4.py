"""Config 4 parity (1024 x 52-card proofs, 128 per GPU), at the
per-GPU share bench.py measures: lockstep batches of 128 proofs, 8 batches in
flight on 8 contexts driven by 8 host threads.  Sampled proofs and their V
commitments are compared byte-for-byte with the serial C prover
(oracle/c/perm_cpu.c, an independent implementation of the same sound-mode
protocol over dalek-style MSMs and bulletproofs' folding IPA); every batch
batch-verifies, and a batch with one tampered proof is rejected.

Reference: circuit_lib.rs:139-476 (create -> blinding_values) and :478-585
(verify); north_star: "outputs are bit-exact".
"""
import threading

import pytest

from oracle import cport

pytestmark = pytest.mark.gpu

K = 52
B = 128
S = 8


def _seeds(b):
    return [7_000_000 + 1000 * b + i for i in range(B)]


def _check_sample(seeds, proofs, Vs, picks):
    for i in picks:
        cpf, cV = cport.cpu_prove(K, seeds[i])
        assert proofs[i] == cpf, f"proof of seed {seeds[i]} differs from the C prover"
        assert Vs[i] == b"".join(cV), f"V of seed {seeds[i]} differs from the C prover"


def test_config4_eight_batches_in_flight_bit_exact():
    import bpperm
    ctxs = [bpperm.Context(0) for _ in range(S)]
    gens = bpperm.Gens(ctxs[0], 128)  # one resident generator set, as bench.py
    provers = [bpperm.PermProver(gens, K, ctx=c) for c in ctxs]
    out = [None] * S
    errs = []

    def run(s):
        try:
            out[s] = provers[s].prove_batch(_seeds(s))
        except Exception as e:  # surfaced after the join
            errs.append(e)

    th = [threading.Thread(target=run, args=(s,)) for s in range(S)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for s in range(S):
        proofs, Vs = out[s]
        assert len(proofs) == B and all(len(p) == provers[s].proof_len for p in proofs)
        # first, last, a lockstep-group border and one more per batch: 4 x 8 = 32 proofs
        _check_sample(_seeds(s), proofs, Vs, [0, 7, 8 + 13 * s % 100, B - 1])
        assert provers[s].verify_batch(proofs, Vs)
    # tampered: one bit of one proof's t_hat in batch 3
    proofs, Vs = out[3]
    bad = list(proofs)
    b = bytearray(bad[77])
    b[8 * 32 + 2 * 32 + 5] ^= 0x10
    bad[77] = bytes(b)
    assert not provers[3].verify_batch(bad, Vs)
    # swapped V vectors between two proofs
    Vbad = list(Vs)
    Vbad[10], Vbad[11] = Vbad[11], Vbad[10]
    assert not provers[3].verify_batch(proofs, Vbad)
    gens.close()
    for c in ctxs:
        c.close()


def test_bench_shape_384_proof_batches_in_flight_bit_exact():
    """bench.py's proofs leg shape: 384-proof lockstep batches, several in
    flight on their own contexts and host threads over one shared generator
    set.  Sampled proofs and V byte-exact against the serial C prover (first,
    last, the 8-way lockstep group borders, the 128 / 256 borders of the
    direct-table launch shapes); every batch verifies; one tampered proof and
    one swapped V are rejected."""
    import bpperm
    B4, S4 = 384, 4
    seeds = [[8_000_000 + 10_000 * s + i for i in range(B4)] for s in range(S4)]
    ctxs = [bpperm.Context(0) for _ in range(S4)]
    gens = bpperm.Gens(ctxs[0], 128)
    provers = [bpperm.PermProver(gens, K, ctx=c) for c in ctxs]
    out = [None] * S4
    errs = []

    def run(s):
        try:
            out[s] = provers[s].prove_batch(seeds[s])
        except Exception as e:  # surfaced after the join
            errs.append(e)

    th = [threading.Thread(target=run, args=(s,)) for s in range(S4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for s in range(S4):
        proofs, Vs = out[s]
        assert len(proofs) == B4 and all(len(p) == provers[s].proof_len for p in proofs)
        picks = [0, 7, 8, 127, 128, 255, 256, 300 + 11 * s, B4 - 1] if s == 0 else [0, 129 + 17 * s, B4 - 1]
        _check_sample(seeds[s], proofs, Vs, picks)
        assert provers[s].verify_batch(proofs, Vs)
    proofs, Vs = out[2]
    bad = list(proofs)
    b = bytearray(bad[333])
    b[8 * 32 + 2 * 32 + 9] ^= 0x04
    bad[333] = bytes(b)
    assert not provers[2].verify_batch(bad, Vs)
    Vbad = list(Vs)
    Vbad[200], Vbad[201] = Vbad[201], Vbad[200]
    assert not provers[2].verify_batch(proofs, Vbad)
    gens.close()
    for c in ctxs:
        c.close()


def test_changing_batch_shapes_on_one_context(ctx):
    """The per-context upload caches (generator indices, circuit CSR, MSM
    offsets: ctx_h2d_const / upload_offsets) see batch sizes 41 -> 128 -> 41
    -> 1 -> 128 on one context; every batch must still match the C prover."""
    import bpperm
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, K)
    for n, base in ((41, 100), (128, 200), (41, 300), (1, 400), (128, 500)):
        seeds = [base * 1000 + i for i in range(n)]
        proofs, Vs = pr.prove_batch(seeds)
        _check_sample(seeds, proofs, Vs, sorted({0, n // 2, n - 1}))
        assert pr.verify_batch(proofs, Vs)
    # a different circuit size on the same context in between
    pr8 = bpperm.PermProver(g, 8)
    proofs, Vs = pr8.prove_batch([1, 2, 3])
    assert pr8.verify_batch(proofs, Vs)
    proofs, Vs = pr.prove_batch([900_000 + i for i in range(41)])
    _check_sample([900_000 + i for i in range(41)], proofs, Vs, [0, 40])
    g.close()


def test_sub_batches_on_child_streams_fresh_gens(monkeypatch):
    """bpp_perm_prove_batch with BPP_PROVE_STREAMS=2 on a freshly created gens:
    the first-use window / direct tables are built once, under the gens lock,
    and published only after their stream finished (gens_points), so the
    child streams never read a half-built table."""
    import bpperm
    monkeypatch.setenv("BPP_PROVE_STREAMS", "2")
    with bpperm.Context(0) as c:
        g = bpperm.Gens(c, 128)
        pr = bpperm.PermProver(g, K)
        seeds = [31_000 + i for i in range(64)]
        proofs, Vs = pr.prove_batch(seeds)
        _check_sample(seeds, proofs, Vs, [0, 31, 32, 63])
        assert pr.verify_batch(proofs, Vs)
        g.close()


def test_shared_fresh_gens_across_threads():
    """Two contexts on two host threads share ONE freshly created gens and
    trigger its first-use table build at the same time."""
    import bpperm
    owner = bpperm.Context(0)
    others = [bpperm.Context(0) for _ in range(2)]
    g = bpperm.Gens(owner, 128)
    out = [None, None]
    errs = []

    def run(s):
        try:
            pr = bpperm.PermProver(g, K, ctx=others[s])
            out[s] = pr.prove_batch([55_000 + 100 * s + i for i in range(16)])
        except Exception as e:
            errs.append(e)

    th = [threading.Thread(target=run, args=(s,)) for s in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for s in range(2):
        seeds = [55_000 + 100 * s + i for i in range(16)]
        _check_sample(seeds, out[s][0], out[s][1], [0, 15])
    g.close()
    for c in others + [owner]:
        c.close()


@pytest.mark.parametrize("k,nb", [(8, 128), (24, 130)])
def test_two_sided_ipa_rounds_other_circuit_sizes(ctx, k, nb):
    """Batches of >= 128 proofs run each IPA round as one block per instance
    walking both L and R (ipa.hip ipa_round_body S = 2).  Other circuit sizes
    than the bench's: k = 8 (n_p = 16, ~2 terms a lane) and k = 24 (n_p =
    64) with an odd batch of 130; sampled proofs byte-exact against the C
    prover, the batch verifies."""
    import bpperm
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, k)
    seeds = [61_000 + 1000 * k + i for i in range(nb)]
    proofs, Vs = pr.prove_batch(seeds)
    for i in sorted({0, 1, 63, 64, nb // 2, nb - 2, nb - 1}):
        cpf, cV = cport.cpu_prove(k, seeds[i])
        assert proofs[i] == cpf, f"proof {i} (k = {k}) differs from the C prover"
        assert Vs[i] == b"".join(cV)
    assert pr.verify_batch(proofs, Vs)
    g.close()
