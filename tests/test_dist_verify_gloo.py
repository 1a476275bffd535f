"""World-size-2 gloo test of the multi-GPU batch verifier (CPU only).

The product's host phase runs on every rank: bpp_perm_verify_begin parses
and replays the transcripts of the rank's proofs; rank 0 draws the batch's
verifier seed and sends it to every rank (bpperm.dist.shared_seed, the one
exchange before the partials); bpp_perm_verify_scalars builds the rank's
weighted MSM terms (every proof's weight mixes the seed with its own r).  Only the MSM itself (bpp_perm_verify_partial on
a GPU) is replaced here by the oracle, so partition + exchange + combine
(bpp_partials_is_identity) are checked end to end without a GPU, for both
splits of SURVEY.md §8(e):

* proof split: rank r holds proofs [first, first + count), all windows;
* window split (north_star): every rank holds every proof, windows
  window_ranges(W, world)[rank];
* sharded window split: rank r expands its slice only, the slices' scalars
  and points are all-gathered, then windows window_ranges(W, world)[rank].

Proofs come from the serial C prover (oracle/c/perm_cpu.c, byte-equal to the
GPU prover in tests/test_gpu_perm.py).  Reference: verify,
circuit_lib.rs:478-585."""
import os
import socket

import pytest
import torch.multiprocessing as mp

K = 2
COUNT = 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tamper, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bulletproof-perm_amd"))
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bpperm
    from bpperm import dist as bdist
    from oracle import cport
    from oracle import ristretto as r255
    from oracle.merlin import bulletproof_gens, pedersen_gens_default

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        proofs, Vs = [], []
        for s in range(COUNT):
            pf, V = cport.cpu_prove(K, 100 + s)
            if tamper and s == 3:  # t_hat + 1 (still canonical): must be rejected
                t = int.from_bytes(pf[8 * 32 + 64: 8 * 32 + 96], "little")
                pf = pf[:8 * 32 + 64] + ((t + 1) % r255.L).to_bytes(32, "little") + pf[8 * 32 + 96:]
            proofs.append(pf)
            Vs.append(b"".join(V))
        n_p = 4
        G, H = bulletproof_gens(n_p)
        B, Bb = pedersen_gens_default()
        gens = list(G) + list(H) + [B, Bb]

        def partial(job, seed, first, wb=None, we=None):
            sc, pts = job.scalars(seed, first)
            s_int = [int.from_bytes(x, "little") for x in sc]
            P = gens + [r255.decode(p) for p in pts]
            if wb is None:
                return r255.raw_point_bytes(r255.msm(s_int, P))
            c, W = job.windows()
            return r255.raw_point_bytes(r255.msm_window_partial(s_int, P, c, W, wb, we))

        seed = bdist.shared_seed(rank)
        assert bdist.torch_all_gather_bytes(seed) == [seed] * world
        # proof split: this rank's slice, all windows, no exchange before the partials
        b, e = bdist.point_ranges(COUNT, world)[rank]
        job = bpperm.VerifyJob(K, proofs[b:e], Vs[b:e])
        assert job.ok
        ok_split = bpperm.partials_is_identity(bdist.torch_all_gather_bytes(partial(job, seed, b)))
        job.close()

        # window split: every proof on every rank, a window range each
        job = bpperm.VerifyJob(K, proofs, Vs)
        c, W = job.windows()
        wb, we = bdist.window_ranges(W, world)[rank]
        ok_win = bpperm.partials_is_identity(bdist.torch_all_gather_bytes(partial(job, seed, 0, wb, we)))
        job.close()

        # sharded window split (bdist.verify_sliced's exchange): each rank
        # expands its slice only; the slices' scalars (generator part summed,
        # proof-point part concatenated) and decoded points are all-gathered,
        # then each rank takes its window range of the whole batch's MSM
        job = bpperm.VerifyJob(K, proofs[b:e], Vs[b:e])
        sc, pts = job.scalars(seed, b)
        job.close()
        NG = 2 * n_p + 2
        blob = b"".join(sc) + b"".join(pts)
        blobs = bdist.torch_all_gather_bytes_var(blob)
        gen_sum = [0] * NG
        s_all, p_all = [], []
        for bl in blobs:
            n_t = len(bl) // 64 - NG // 2  # (scalar count = NG + points; the blob holds both, 32 B each)
            sc_r = [bl[32 * i: 32 * i + 32] for i in range(NG + n_t)]
            pts_r = [bl[32 * (NG + n_t) + 32 * i: 32 * (NG + n_t) + 32 * i + 32] for i in range(n_t)]
            gen_sum = [(a + int.from_bytes(x, "little")) % r255.L for a, x in zip(gen_sum, sc_r[:NG])]
            s_all += [int.from_bytes(x, "little") for x in sc_r[NG:]]
            p_all += pts_r
        c, W = bpperm.msm_windows(NG + len(p_all))
        assert W == bdist._batch_windows(K, COUNT)
        wb, we = bdist.window_ranges(W, world)[rank]
        P = gens + [r255.decode(p) for p in p_all]
        part = r255.raw_point_bytes(r255.msm_window_partial(gen_sum + s_all, P, c, W, wb, we))
        ok_shard = bpperm.partials_is_identity(bdist.torch_all_gather_bytes(part))
        q.put((rank, ok_split, ok_win, ok_shard))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tamper", [False, True])
def test_verify_split_over_gloo(tamper):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, tamper, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    results = sorted(q.get() for _ in range(world))
    for _, ok_split, ok_win, ok_shard in results:
        assert ok_split == (not tamper)
        assert ok_win == (not tamper)
        assert ok_shard == (not tamper)


def test_verify_job_host_phase_matches_oracle():
    """The product's host replay + weighting, fed to the oracle's MSM, gives
    the identity for honest proofs; a malformed proof fails in begin."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bulletproof-perm_amd"))
    sys.path.insert(0, str(root))
    import bpperm
    from oracle import cport
    from oracle import ristretto as r255
    from oracle.merlin import bulletproof_gens, pedersen_gens_default

    proofs, Vs = zip(*[cport.cpu_prove(K, 7 + s) for s in range(3)])
    Vs = [b"".join(v) for v in Vs]
    job = bpperm.VerifyJob(K, proofs, Vs)
    assert job.ok and len(job.r) == 96
    T = job.terms()
    assert T == 2 * 4 + 2 + 3 * (2 * K + 1 + 8 + 2 * 2)
    G, H = bulletproof_gens(4)
    B, Bb = pedersen_gens_default()
    seed = bpperm.verify_seed()
    sc, pts = job.scalars(seed, 0)
    P = list(G) + list(H) + [B, Bb] + [r255.decode(p) for p in pts]
    assert r255.equal(r255.msm([int.from_bytes(x, "little") for x in sc], P), r255.IDENTITY)
    # the same job as batch proofs 5..7: other weights, still the identity
    sc2, _ = job.scalars(seed, 5)
    assert sc2 != sc
    assert r255.equal(r255.msm([int.from_bytes(x, "little") for x in sc2], P), r255.IDENTITY)
    job.close()
    # A_I = the identity encoding: validate_and_append_point rejects it
    # (transcript_protocol.rs:48-60); undecodable points fail later, in the
    # GPU decompression of bpp_perm_verify_partial
    bad = bytes(32) + proofs[1][32:]
    job = bpperm.VerifyJob(K, [proofs[0], bad], Vs[:2])
    assert not job.ok
