"""Per-rank phase times of the upload-sharded window split (bpperm.dist.
verify_sliced) on ONE GPU, for the N = 8 model in DESIGN.md §5: rank 0's own
work at world N as verify_sliced orders it -- the asynchronous begin of its
slice job ("job": staging + upload enqueue of count / N proofs), its point
block ("points": until the decompression is done; the points' all-gather
starts here), its scalar block ("scalars": until the replay and the scalar
expansion are done), and the MSM of the whole batch over its window range -- with the all-gathers replaced by
device-local blocks (the xGMI transfer is modelled from the bytes printed).

    python tools/shard_model.py [--proofs 4096] [--reps 5] [--worlds 1,2,4,8]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

SEED = bytes(range(32))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proofs", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--k", type=int, default=52)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--no-proof-split", action="store_true",
                    help="skip the proof split's rank 0 (a trace then ends with the sharded partial)")
    a = ap.parse_args()
    import bpperm
    from bpperm import dist as bdist
    ctx = bpperm.Context(0)
    g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, a.k)
    proofs, Vs = [], []
    for b in range(0, a.proofs, 256):
        p, v = pr.prove_batch(list(range(900_000 + b, 900_000 + min(a.proofs, b + 256))))
        proofs += p
        Vs += v
    W = bdist._batch_windows(a.k, a.proofs)
    out = {"proofs": a.proofs, "windows": W, "worlds": {}}
    for world in [int(x) for x in a.worlds.split(",")]:
        ranges = bdist.point_ranges(a.proofs, world)
        counts = [e - b for b, e in ranges]
        stride = (bdist._slice_block_bytes(a.k, max(counts)) + 15) // 16 * 16
        pstride = max(counts) * bdist._points_per_proof(a.k) * 128
        blocks = ctx.dev_alloc(world * stride)
        pblocks = ctx.dev_alloc(world * pstride)
        # the other ranks' blocks (untimed): their jobs run on this context in turn
        for r in range(1, world):
            b, e = ranges[r]
            j = bpperm.VerifyJob(a.k, proofs[b:e], Vs[b:e], pr.label, ctx=ctx)
            assert j.ok and j.slice_points(pblocks + r * pstride)
            j.slice_scalars(SEED, blocks + r * stride, first=b)
            j.close()
        b, e = ranges[0]
        wb, we = bdist.window_ranges(W, world)[0]
        t = {"job": [], "points": [], "scalars": [], "partial": []}
        for rep in range(a.reps + 1):
            tj = time.perf_counter()
            b"".join(proofs[b:e]), b"".join(Vs[b:e])  # (VerifyJob's own joins, taken out of "job")
            tj = time.perf_counter() - tj
            t0 = time.perf_counter()
            j = bpperm.VerifyJob(a.k, proofs[b:e], Vs[b:e], pr.label, ctx=ctx, wait=False)
            t1 = time.perf_counter() - tj
            assert j.ok and j.slice_points(pblocks)
            t2 = time.perf_counter()
            assert j.slice_scalars(SEED, blocks, first=0)
            t3 = time.perf_counter()
            part = pr.verify_partial_sharded(j, 0, blocks, stride, pblocks, pstride, counts, wb, we)
            t4 = time.perf_counter()
            j.close()
            if rep:
                for k, v in zip(t, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                    t[k].append(v * 1e3)
        # the proof split's rank 0: its slice job and the MSM of its slice over all windows
        t["proofs_split"] = []
        for rep in range(0 if a.no_proof_split else a.reps + 1):
            t0 = time.perf_counter()
            j = bpperm.VerifyJob(a.k, proofs[b:e], Vs[b:e], pr.label, ctx=ctx, wait=False)
            _, Wj = j.windows()
            part_p = pr.verify_partial(j, SEED, b, 0, Wj)
            t1 = time.perf_counter()
            j.close()
            assert part_p is not None
            if rep:
                t["proofs_split"].append((t1 - t0) * 1e3)
        med = {k: round(sorted(v)[len(v) // 2], 4) for k, v in t.items() if v}
        out["worlds"][world] = {"slice_proofs": counts[0], "window_range": [wb, we], "ms": med,
                                "gather_bytes_per_rank": {"points": pstride * (world - 1), "scalars": stride * (world - 1)},
                                "partial_nonzero": part != bytes(128)}
        ctx.dev_free(blocks)
        ctx.dev_free(pblocks)
    print(json.dumps(out))
    g.close()
    ctx.close()


if __name__ == "__main__":
    main()
