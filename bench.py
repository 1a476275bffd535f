#!/usr/bin/env python3
"""bench.py — Ristretto MSM pairs/s on MI355X (+ CPU baseline, roofline).

Metric (BASELINE.json): "permutation proofs/sec + Ristretto MSM pairs/sec at
1/2/4/8 MI355X".  `value` is MSM scalar-point pairs/s of one step = one full
multiscalar multiplication over synthetic uniform scalars and distinct
hash-to-group points already resident in HBM (2^20
pairs on one GPU).  At N GPUs the MSM has 2^20*N pairs and its bucket
windows are partitioned across the ranks (config 5 shape: 2^22 at N=4); each
rank computes the partial sum of its windows and the 128-byte partial points
are all-gathered over RCCL and added (RCCL cannot add curve points), so
per-GPU work is fixed: "scaling": "weak".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--log2n 20]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))

L = 2**252 + 27742317777372353535851937790883648493
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# Integer-ALU roofline: independent GF(2^255-19) multiplies per second on the
# whole chip with the product's own field code (10-limb radix 2^25.5),
# measured by tools/ubench/felat at 4096 x 64-lane blocks
# (profiles/r01_felat_fe10.txt).  One mixed addition (ge_madd) = 7 field
# multiplies.
FE_MUL_PEAK_GOPS = 273.0


def synth_scalars(n: int, seed: int) -> bytes:
    """Uniform scalars = from_bytes_mod_order_wide(SHAKE256 bytes) (dalek
    Scalar::random shape), serialized canonical little-endian."""
    raw = hashlib.shake_256(b"bench-scalars" + seed.to_bytes(8, "little")).digest(64 * n)
    out = bytearray(32 * n)
    for i in range(n):
        s = int.from_bytes(raw[64 * i: 64 * i + 64], "little") % L
        out[32 * i: 32 * i + 32] = s.to_bytes(32, "little")
    return bytes(out)


def synth_point_bytes(n: int, seed: int) -> bytes:
    """64 uniform bytes per point -> RistrettoPoint::from_uniform_bytes (on GPU)."""
    return hashlib.shake_256(b"bench-points" + seed.to_bytes(8, "little")).digest(64 * n)


def load_traffic(stage: str, log2n: int):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary."""
    p = ROOT / "profiles" / "pmc_summary.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(f"{stage}@2^{log2n}", {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(seconds: float = 12.0):
    """Serial C restatement of dalek-ng's Pippenger (oracle/c, 'port') timed
    on a bounded sample of the same workload: one 2^16-pair MSM, repeated
    until ~`seconds` of CPU time, 1 thread (dalek-ng's serial backend is
    single-threaded).  An all-host-cores figure (one MSM per thread) rides
    along as `all_cores`."""
    try:
        sys.path.insert(0, str(ROOT))
        from oracle import cport
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "pairs/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}
    out = cport.bench_msm(log2n=16, seconds=seconds)
    out["all_cores"] = cport.bench_msm_threads(log2n=16, seconds=seconds / 2, threads=cport.host_cores())
    return out


def cpu_baseline_proofs(seconds: float = 8.0):
    """52-card proofs/s of the serial C prover restatement (oracle/c/perm_cpu.c:
    dalek-style MSMs, bulletproofs' folding IPA, merlin), 1 core and all
    host cores (one proof per thread)."""
    try:
        sys.path.insert(0, str(ROOT))
        from oracle import cport
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "proofs/s", "cores": 1, "kind": "port", "sample": f"unavailable: {e}"}
    out = cport.bench_prove(52, seconds=seconds, threads=1)
    out["all_cores"] = cport.bench_prove(52, seconds=seconds / 2, threads=cport.host_cores())
    return out


def bench_proofs(ctx, args, world, rank, torch, dist, cdev="cuda"):
    """Config 4: batches of 52-card permutation proofs, sharded one batch per
    GPU (independent proofs: no collective on the data path), proved in
    lockstep on each GPU; then the same proofs batch-verified (one MSM per
    batch).  Throughput: `--proof-streams` batches in flight per GPU, each
    driven by its own host thread and context (own HIP stream; ctypes drops
    the GIL), so one batch's host phases (transcripts, challenges) run while
    another's kernels occupy the GPU.  Returns whole-job proofs/s (max time
    over ranks) and the one-batch-at-a-time latency."""
    import threading

    import bpperm
    B = args.proofs_per_gpu
    S = max(1, args.proof_streams)
    ctxs = [ctx] + [bpperm.Context(ctx.device) for _ in range(S - 1)]
    gens = [bpperm.Gens(c, 128) for c in ctxs]
    provers = [bpperm.PermProver(g, 52) for g in gens]

    def seeds(step, s):
        return [(((step * S + s) * world + rank) * B + i) for i in range(B)]

    for s, pr in enumerate(provers):  # warmup (window tables, workspaces)
        pr.prove_batch(seeds(10_000, s))
        pr.prove_batch(seeds(10_001, s))

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=cdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        return out, el

    def in_flight(fn):
        res = [None] * S
        errs = []

        def run(s):
            try:
                res[s] = fn(s)
            except Exception as e:  # surfaced after the join
                errs.append(e)

        th = [threading.Thread(target=run, args=(s,)) for s in range(S)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return res

    # one batch at a time on one stream (latency)
    _, el_one = timed(lambda: [provers[0].prove_batch(seeds(20_000 + st, 0)) for st in range(args.proof_steps)])
    # S batches in flight (throughput)
    batches, el_p = timed(lambda: in_flight(
        lambda s: [provers[s].prove_batch(seeds(st, s)) for st in range(args.proof_steps)]))

    def verify_stream(s):
        ok = True
        for proofs, Vs in batches[s]:
            ok &= provers[s].verify_batch(proofs, Vs)
        return ok

    oks, el_v = timed(lambda: in_flight(verify_stream))
    total = B * S * world * args.proof_steps
    for g in gens:
        g.close()
    for c in ctxs[1:]:
        c.close()
    return {"metric": "52-card permutation proofs/sec (prove)", "value": total / el_p, "unit": "proofs/s",
            "ms_per_batch": el_p / (args.proof_steps * S) * 1e3, "proofs_per_gpu_per_batch": B,
            "batches_in_flight_per_gpu": S, "batches": args.proof_steps * S,
            "latency_ms_per_batch": el_one / args.proof_steps * 1e3,
            "verify_batch_proofs_per_sec": total / el_v, "verify_ms_per_batch": el_v / (args.proof_steps * S) * 1e3,
            "all_verified": bool(all(oks)), "n_gpus": world, "scaling": "weak",
            "config": f"config 4: 52-card sound-mode permutation proofs, lockstep batches of {B} per GPU, "
                      f"{S} batches in flight per GPU (one host thread + context each)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log2n", type=int, default=20, help="pairs per GPU = 2^log2n")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verify", action="store_true", help="also recompute via a second window split")
    ap.add_argument("--proofs-per-gpu", type=int, default=128,
                    help="52-card proofs per GPU per batch (config 4: 1024 over 8 GPUs); 0 = skip")
    ap.add_argument("--proof-steps", type=int, default=16,
                    help="batches per stream (8 streams x 16 = 128 batches, ~0.25 s timed)")
    ap.add_argument("--proof-streams", type=int, default=8, help="proof batches in flight per GPU")
    ap.add_argument("--inflight", type=int, default=3, help="independent MSMs in flight (1..4)")
    ap.add_argument("--msm-split", choices=["windows", "points"], default="windows",
                    help="N>1: split the MSM's bucket windows (default) or its points over the ranks")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    # BPP_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on one
    # GPU (RCCL needs one GPU per rank); the driver's runs use nccl = RCCL.
    backend = os.environ.get("BPP_DIST_BACKEND", "nccl")
    cdev = "cuda" if backend == "nccl" else "cpu"  # device of collective tensors
    if world > 1:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    import bpperm

    n_local = 1 << args.log2n
    n = n_local * world
    ctx = bpperm.Context(local)

    # ---- inputs resident in HBM before the timed region.  The global MSM is
    # the concatenation of `world` slices with per-slice seeds, so both
    # partitions compute the same result (result_prefix agrees).
    t0 = time.time()
    slices = range(world) if args.msm_split == "windows" else [rank]
    pts = ctx.from_uniform(b"".join(synth_point_bytes(n_local, 3 + 1000 * s) for s in slices))
    sc = b"".join(synth_scalars(n_local, 2 + 1000 * s) for s in slices)
    n_here = len(sc) // 32
    d_sc = ctx.dev_alloc(len(sc))
    ctx.htod(d_sc, sc)
    # a second scalar vector: consecutive pipelined MSMs are distinct inputs
    sc2 = b"".join(synth_scalars(n_local, 7 + 1000 * s) for s in slices)
    d_sc2 = ctx.dev_alloc(len(sc2))
    ctx.htod(d_sc2, sc2)
    del sc, sc2
    setup_s = time.time() - t0

    c, W = bpperm.msm_windows(n_here)
    if args.msm_split == "windows":  # contiguous window ranges per rank (north_star's split)
        cuts = [(W * r) // world for r in range(world + 1)]
        wb, we = cuts[rank], cuts[rank + 1]
    else:  # this rank's point slice, all windows
        wb, we = 0, W

    def step():
        if world == 1:
            return ctx.msm_table_dev(d_sc, pts, n)
        part = ctx.msm_table_dev_partial(d_sc, pts, n_here, wb, we)
        t = torch.frombuffer(bytearray(part), dtype=torch.uint8).to(cdev)
        gathered = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        return bpperm.partials_finish([g.cpu().numpy().tobytes() for g in gathered])

    def finish(raw):
        if world == 1:
            return raw
        t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(cdev)
        gathered = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(gathered, t)
        return bpperm.partials_finish([g.cpu().numpy().tobytes() for g in gathered])

    def run_pipelined(k):
        """k MSMs (alternating scalar vectors), --inflight of them in flight
        (3 by default): MSM i+1 is submitted before MSM i is collected, so
        the device sorts i+1 beside i's bucket reduction and the host
        combines i's windows (and, N > 1, all-gathers its partial) while
        the device accumulates i+1."""
        bufs = (d_sc, d_sc2)
        we_ = we if world > 1 else 0
        out, ticks = [], []
        for i in range(k + args.inflight - 1):
            if i < k:
                ticks.append(ctx.msm_submit(bufs[i % 2], pts, n_here, wb, we_))
            if i >= args.inflight - 1:
                out.append(finish(ctx.msm_collect(ticks.pop(0), partial=world > 1)))
        return out

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=cdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = tt.item()
        return r, el

    # one MSM at a time (latency), then the pipelined stream (throughput)
    for _ in range(args.warmup):
        res = step()
    res, el_serial = timed(lambda: [step() for _ in range(args.steps)])
    res = res[-1]
    # (the first stream through fresh child contexts runs ~30 % slow for its
    # first ~25 ms on the box: warm a full-length stream)
    run_pipelined(max(args.steps, 8, args.warmup))
    piped, el = timed(lambda: run_pipelined(args.steps))
    if os.environ.get("BENCH_DEBUG"):
        for _ in range(3):
            t1 = time.perf_counter()
            run_pipelined(args.steps)
            print(f"pipelined again: {(time.perf_counter() - t1) / args.steps * 1e3:.4f} ms", file=sys.stderr)
    pipe_ok = piped[0] == res and (len(piped) < 2 or piped[1] != res)

    # ---- per-kernel timing (HIP events on the library stream), separate pass
    ctx.profile(True)
    ctx.profile_reset()
    prof_steps = max(2, min(args.steps, 5))
    for _ in range(prof_steps):
        if world == 1:
            ctx.msm_table_dev(d_sc, pts, n)
        else:
            ctx.msm_table_dev_partial(d_sc, pts, n_here, wb, we)
    stages = {}
    launches = {}
    for st in ("msm_digits", "msm_count", "msm_scan", "msm_scatter", "msm_accumulate", "msm_fixup", "msm_reduce"):
        ms, k = ctx.profile_get(st)
        stages[st] = ms / max(k, 1)  # per launch
        launches[st] = k / prof_steps  # launches per MSM (one per window group)
    ctx.profile(False)

    proofs = None
    if args.proofs_per_gpu > 0:
        proofs = bench_proofs(ctx, args, world, rank, torch, dist, cdev)

    ms_step = el / args.steps * 1e3
    value = n * args.steps / el
    acc_ms = stages["msm_accumulate"]
    # The MSM runs as window groups (one accumulate launch per group, on two
    # streams): one launch's share of the MSM's algorithmic bytes
    # (32 B scalar + 64 B affine point per pair) and of its n*W
    # mixed additions.
    acc_launches = max(launches["msm_accumulate"], 1.0)
    algo_bytes = 96 * n_here / acc_launches
    madds = n_here * (we - wb) / acc_launches
    achieved = algo_bytes / (acc_ms * 1e-3) / 1e9 if acc_ms > 0 else None

    line = {
        "metric": "Ristretto MSM scalar-point pairs/sec",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "latency_ms_per_msm": el_serial / args.steps * 1e3,
        "pipelined_matches_serial": bool(pipe_ok),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 limbs (GF(2^255-19) integer)",
        "data": "synthetic: uniform scalars (SHAKE256 -> mod l), hash-to-group points (from_uniform_bytes on GPU)",
        "config": {"workload": f"ristretto255 Pippenger MSM, 2^{args.log2n} pairs per GPU (config 3; config 5 shape at N=4)",
                   "pairs": n, "window_bits": c, "windows": W,
                   "parallelism": f"{'window' if args.msm_split == 'windows' else 'point'}-partition x{world}",
                   "in_flight": f"{args.inflight} independent MSMs (bpp_msm_submit/collect); latency_ms_per_msm is one at a time"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                     "traffic": load_traffic("msm_accumulate", args.log2n),
                     "kernel": "k_msm_accumulate", "kernel_ms": acc_ms,
                     "algo_bytes_per_launch": algo_bytes, "launches_per_msm": acc_launches},
        "alu_roofline": {"achieved": (7 * madds / (acc_ms * 1e-3) / 1e9) if acc_ms > 0 else None,
                         "peak": FE_MUL_PEAK_GOPS, "unit": "G field-mul/s",
                         "frac": (7 * madds / (acc_ms * 1e-3) / 1e9 / FE_MUL_PEAK_GOPS) if acc_ms > 0 else None,
                         "note": "k_msm_accumulate: (pairs x windows) mixed additions per launch x 7 field multiplies"},
        "stage_ms": stages,
        "proofs": proofs,
        "setup_s": setup_s,
        "result_prefix": res.hex()[:16],
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        if proofs is not None:
            proofs["cpu_baseline"] = cpu_baseline_proofs()
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.dev_free(d_sc)
    ctx.dev_free(d_sc2)
    pts.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
