"""World-size-2 gloo test of the multi-GPU MSM partition (CPU only).

Each rank computes the partial sum of its bucket-window range (the same
bpperm.dist.window_ranges split bench.py uses over RCCL), the 128-byte raw
partials are all-gathered over gloo, and bpp_partials_finish (host code of
libbpperm, no GPU) adds them.  The per-rank partial is computed by the
oracle's restatement of the GPU digit recoding, so this checks the
partition + exchange + combine logic end to end without a GPU."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "bulletproof-perm_amd"))
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bpperm
    from bpperm import dist as bdist
    from oracle import ristretto as r255
    from oracle.merlin import Rng

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = Rng(42, b"dist-test")
        pts = [rng.point() for _ in range(n)]
        sc = [rng.scalar() for _ in range(n)]
        c, W = bpperm.msm_windows(n)

        def partial(wb, we):
            return r255.raw_point_bytes(r255.msm_window_partial(sc, pts, c, W, wb, we))

        res = bdist.distributed_msm(partial, W, rank, world, bdist.torch_all_gather_bytes, bpperm.partials_finish)
        want = r255.encode(r255.msm(sc, pts))

        def partial_pts(b, e):  # alternative split: points, all windows
            return r255.raw_point_bytes(r255.msm(sc[b:e], pts[b:e]))

        res2 = bdist.distributed_msm_points(partial_pts, n, rank, world, bdist.torch_all_gather_bytes,
                                            bpperm.partials_finish)
        q.put((rank, res == want and res2 == want, bdist.window_ranges(W, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_window_partition_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 24, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    results = sorted(q.get() for _ in range(world))
    assert all(ok for _, ok, _ in results)
    ranges = results[0][2]
    assert ranges[0][0] == 0 and ranges[-1][1] > ranges[0][1]


def test_window_ranges_cover_exactly():
    from bpperm.dist import window_ranges, shard_proofs
    for W in (1, 5, 16, 19, 33):
        for world in (1, 2, 3, 4, 8):
            rs = window_ranges(W, world)
            assert rs[0][0] == 0 and rs[-1][1] == W
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
    owned = sorted(i for r in range(4) for i in shard_proofs(10, r, 4))
    assert owned == list(range(10))
