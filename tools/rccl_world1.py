"""bpperm.dist's collective paths over RCCL (torch.distributed "nccl") on
ONE GPU: a world-1 process group, so every RCCL call bench.py's N > 1 legs
make -- all_gather of the 128-B MSM partials and of the ok flags, the
verifier seed's all-gather, all_gather_into_tensor of the sharded split's
point and scalar blocks, the MAX all_reduce of the timings -- runs on the
device through RCCL, with the exact-result checks of the gloo tests.
Prints one JSON line; exit status 0 = every check passed.

    python tools/rccl_world1.py [--port P]
"""
import argparse
import hashlib
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=29531)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{a.port}", rank=0, world_size=1)
    import bpperm
    from bpperm import dist as bdist
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    ctx = bpperm.Context(0)
    # MSM window split: the partial of every window, all-gathered over RCCL
    n = 1 << 16
    pts = ctx.from_uniform(hashlib.shake_256(b"rccl-pts").digest(64 * n))
    raw = bytearray(hashlib.shake_256(b"rccl-sc").digest(32 * n))
    raw[31::32] = bytes(n)  # < 2^248: canonical
    d_sc = ctx.dev_alloc(32 * n)
    ctx.htod(d_sc, bytes(raw))
    c, W = bpperm.msm_windows(n)
    got = bdist.distributed_msm(lambda wb, we: ctx.msm_table_dev_partial(d_sc, pts, n, wb, we), W, 0, 1,
                                lambda b: bdist.torch_all_gather_bytes(b, "cuda"), bpperm.partials_finish)
    out["msm_window_split_ok"] = got == ctx.msm_table_dev(d_sc, pts, n)
    ctx.dev_free(d_sc)
    pts.close()
    # config-5 batch verification, all three splits, and the config-4 job's
    # verification of the rank's own proofs
    gens = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(gens, 52, ctx=ctx)
    proofs, Vs = pr.prove_batch(list(range(1000, 1064)))
    bad = list(proofs)
    b = bytearray(bad[17])
    b[8 * 32 + 70] ^= 1
    bad[17] = bytes(b)
    for split in ("windows", "windows_sharded", "proofs"):
        out[f"{split}_accepts"] = bdist.distributed_verify(pr, proofs, Vs, 0, 1, split, "cuda")
        out[f"{split}_rejects"] = not bdist.distributed_verify(pr, bad, Vs, 0, 1, split, "cuda")
    out["own_slice_accepts"] = bdist.verify_own_slice(pr, proofs, Vs, 0, 0, 1, "cuda")
    out["own_slice_rejects"] = not bdist.verify_own_slice(pr, bad, Vs, 0, 0, 1, "cuda")
    # bench.py's timing reduction
    t = torch.tensor([1.5], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out["all_reduce_ok"] = t.item() == 1.5
    gens.close()
    ctx.close()
    dist.destroy_process_group()
    out["ok"] = all(v for k, v in out.items() if k.endswith(("_ok", "_accepts", "_rejects")))
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
