"""Multi-GPU partitions run end to end through the PRODUCT on the GPU: two
ranks (spawned processes sharing cuda:0, gloo collectives standing in for
RCCL) each compute their share with libbpperm and exchange the 128-byte
partials, exactly as bench.py's N > 1 path does over RCCL.

* the large MSM split by bucket windows (bpp_msm_table_dev_partial over the
  rank's window range) and by points (each rank's slice, all windows):
  bpp_partials_finish of the gathered partials == the serial C port of
  dalek's MSM (oracle/c) on the same inputs, bit-exact;
* the batch verifier split by windows and by proofs
  (bpperm.dist.distributed_verify -> bpp_perm_verify_partial): accepts a
  valid batch and rejects one with a tampered proof on every rank
  (circuit_lib.rs:478-585 in sound form)."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
LOGN = 16
NPROOFS = 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    from oracle import ristretto as r255
    n = 1 << LOGN
    raw = hashlib.shake_256(b"gpu-dist-points").digest(64 * n)
    sraw = hashlib.shake_256(b"gpu-dist-scalars").digest(64 * n)
    sc = b"".join((int.from_bytes(sraw[64 * i: 64 * i + 64], "little") % r255.L).to_bytes(32, "little")
                  for i in range(n))
    return n, raw, sc


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bulletproof-perm_amd"))
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bpperm
    from bpperm import dist as bdist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        with bpperm.Context(0) as ctx:
            n, raw, sc = _inputs()
            # window split: every rank holds every point, a window range each
            tbl = ctx.from_uniform(raw)
            d = ctx.dev_alloc(32 * n)
            ctx.htod(d, sc)
            c, W = bpperm.msm_windows(n)
            out["windows"] = bdist.distributed_msm(lambda wb, we: ctx.msm_table_dev_partial(d, tbl, n, wb, we), W,
                                                   rank, world, bdist.torch_all_gather_bytes, bpperm.partials_finish)
            ctx.dev_free(d)
            tbl.close()
            # point split: each rank its slice of points, all windows
            b, e = bdist.point_ranges(n, world)[rank]
            t2 = ctx.from_uniform(raw[64 * b: 64 * e])
            d2 = ctx.dev_alloc(32 * (e - b))
            ctx.htod(d2, sc[32 * b: 32 * e])
            _, W2 = bpperm.msm_windows(e - b)
            part = ctx.msm_table_dev_partial(d2, t2, e - b, 0, W2)
            out["points"] = bpperm.partials_finish(bdist.torch_all_gather_bytes(part))
            ctx.dev_free(d2)
            t2.close()
            # batch verification split (every rank proves the same seeds)
            g = bpperm.Gens(ctx, 128)
            pr = bpperm.PermProver(g, 52)
            proofs, Vs = pr.prove_batch(list(range(500, 500 + NPROOFS)))
            proofs, Vs = list(proofs), list(Vs)
            for split in ("windows", "proofs"):
                out[f"verify_{split}"] = bdist.distributed_verify(pr, proofs, Vs, rank, world, split)
            bad = bytearray(proofs[5])
            bad[8 * 32 + 40] ^= 1  # a low byte of mu (after the 8 points and tau_x): must fail
            proofs[5] = bytes(bad)
            for split in ("windows", "proofs"):
                out[f"reject_{split}"] = not bdist.distributed_verify(pr, proofs, Vs, rank, world, split)
            g.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_ranks_msm_and_verify_splits():
    from oracle import cport
    world = 2
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    n, raw, sc = _inputs()
    want = cport.msm(sc, cport.from_uniform(raw))
    for rank in range(world):
        r = results[rank]
        assert r["windows"] == want, f"rank {rank}: window split != C port"
        assert r["points"] == want, f"rank {rank}: point split != C port"
        assert r["verify_windows"] and r["verify_proofs"], f"rank {rank}: valid batch rejected"
        assert r["reject_windows"] and r["reject_proofs"], f"rank {rank}: tampered batch accepted"
