"""Multi-GPU partitioning for the two parallel shapes of SURVEY.md §8(e).

1. One large MSM (configs 3/5): the W bucket windows of the signed
   radix-2^c decomposition are split into contiguous ranges, one per rank.
   Each rank runs the full Pippenger pipeline for its windows only and
   produces a raw extended partial point (128 bytes).  RCCL cannot add curve
   points (ncclSum is integer/float), so the exchange is an all_gather of
   the 128-byte partials followed by an exact EC addition on every rank
   (bpp_partials_finish).  Payload: world x 128 B per MSM.

   Alternative (SURVEY.md §8e asks to benchmark both): split the POINTS,
   N/world per rank; every rank runs all W windows over its slice and the
   same 128-byte partial exchange follows (bench.py --msm-split points).

2. Independent proofs (config 4): proof i -> rank i mod world; no
   collective on the data path.

3. Batch verification (config 5): the weighted checks of all proofs form
   ONE MSM (bpp_perm_verify_*).  The batch weights mix a 32-byte verifier
   seed (drawn on rank 0 and sent to every rank, shared_seed) with each
   proof's own transcript challenge r, so no rank needs another rank's
   proofs or challenges.  Window split (north_star): every rank replays
   every proof (on its GPU) and runs its window range; the 128-byte partials
   are all-gathered and must add up to the identity.  Proof split: each
   rank replays its slice and runs all windows of its slice's MSM -- no
   exchange before the 128-byte partials.  Sharded window split
   ("windows_sharded", VERDICT r3/r4: the plain window split uploads,
   decompresses, replays and expands every proof on every rank): every rank
   uploads, decompresses, replays and expands only its proof slice, writes
   its slice's decompressed points (128 B each) and MSM scalars (generator
   scalars summed over the slice, then the slice's proof-point scalars) to
   two device blocks, both are all-gathered (RCCL all_gather_into_tensor over
   xGMI: 70 MB of points and 16.7 MB of scalars in all for config 5), and
   each rank runs the MSM of the whole batch over its window range.

The functions take the collective as a callable so the same code runs over
RCCL on GPUs (bench.py) and over gloo on CPU (tests/test_dist_gloo.py).
"""
from __future__ import annotations

from typing import Callable, Sequence


def window_ranges(W: int, world: int) -> list[tuple[int, int]]:
    """Contiguous, near-equal window ranges [wb, we) for each rank."""
    cuts = [(W * r) // world for r in range(world + 1)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def distributed_msm(partial_fn: Callable[[int, int], bytes], W: int, rank: int, world: int,
                    all_gather: Callable[[bytes], Sequence[bytes]], finish: Callable[[Sequence[bytes]], bytes]) -> bytes:
    """partial_fn(wb, we) -> 128-byte raw partial for this rank's windows;
    all_gather(bytes) -> list of every rank's bytes; finish(partials) ->
    compressed 32-byte result."""
    wb, we = window_ranges(W, world)[rank]
    part = partial_fn(wb, we)
    assert len(part) == 128
    return finish(all_gather(part))


def point_ranges(n: int, world: int) -> list[tuple[int, int]]:
    """Contiguous, near-equal point (term) ranges [b, e) for each rank."""
    cuts = [(n * r) // world for r in range(world + 1)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def distributed_msm_points(partial_fn: Callable[[int, int], bytes], n: int, rank: int, world: int,
                           all_gather: Callable[[bytes], Sequence[bytes]],
                           finish: Callable[[Sequence[bytes]], bytes]) -> bytes:
    """partial_fn(b, e) -> 128-byte raw MSM over terms [b, e) (all windows)."""
    b, e = point_ranges(n, world)[rank]
    part = partial_fn(b, e)
    assert len(part) == 128
    return finish(all_gather(part))


def shard_proofs(count: int, rank: int, world: int) -> list[int]:
    """Proof indices owned by `rank` (round-robin, config 4)."""
    return list(range(rank, count, world))


def torch_all_gather_bytes(payload: bytes, device=None) -> list[bytes]:
    """all_gather of a fixed-size byte payload over the default process group
    (RCCL when the group backend is nccl and device is a GPU, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    t = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().numpy().tobytes() for o in out]


def torch_all_gather_bytes_var(payload: bytes, device=None) -> list[bytes]:
    """all_gather of per-rank payloads of different lengths (sizes first,
    then the payloads padded to the longest)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(x.item()) for x in sizes]
    mx = max(max(sizes), 1)
    t = torch.zeros(mx, dtype=torch.uint8)
    if payload:
        t[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().numpy().tobytes()[:sz] for o, sz in zip(out, sizes)]


def _slice_block_bytes(k: int, count: int) -> int:
    """Bytes of one slice's scalar block (bpp_perm_verify_slice_bytes)."""
    n_p = 1
    while n_p < 2 * k:
        n_p <<= 1
    lg = n_p.bit_length() - 1
    return (2 * n_p + 2 + count * (2 * k + 1 + 8 + 2 * lg)) * 32


def gather_blocks(block, world: int, device=None):
    """all_gather of equal-size uint8 device tensors into one device tensor
    [world * len(block)]: all_gather_into_tensor over RCCL, through host
    memory over gloo."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return block
    if dist.get_backend() == "nccl":
        out = torch.empty(world * block.numel(), dtype=torch.uint8, device=block.device)
        dist.all_gather_into_tensor(out, block)
        return out
    parts = [torch.empty(block.numel(), dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(parts, block.cpu())
    return torch.cat(parts).to(block.device)


def shared_seed(rank: int, device=None) -> bytes:
    """The batch's 32-byte verifier seed, drawn on rank 0 (bpp_verify_seed)
    and sent to every rank -- the one exchange a split batch verification
    needs before its MSM partials (the weights need nothing from the other
    ranks' proofs)."""
    import bpperm

    mine = bpperm.verify_seed() if rank == 0 else bytes(32)
    return torch_all_gather_bytes(mine, device)[0]


def verify_sliced(prover, proofs, Vs, rank: int, world: int, seed: bytes, gather, device=None):
    """The sharded window split of one batch (module doc, 3): returns (ok,
    this rank's 128-B partial).  seed = the batch's verifier seed (the same
    on every rank); gather(block tensor) -> the blocks of all ranks as one
    device tensor (rank order)."""
    import torch

    import bpperm

    ranges = point_ranges(len(proofs), world)
    b, e = ranges[rank]
    counts = [hi - lo for lo, hi in ranges]
    stride = (_slice_block_bytes(prover.k, max(counts)) + 15) // 16 * 16
    pstride = max(counts) * _points_per_proof(prover.k) * 128
    # (the blocks live on the library context's GPU whatever device the
    # collectives use; ADVICE r4: not torch's current device)
    dev = torch.device("cuda", prover.ctx.device)
    blk = torch.zeros(stride, dtype=torch.uint8, device=dev)
    pblk = torch.zeros(pstride, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)  # (the fills run on torch's stream, the library on its own)
    # this rank's slice only: its upload, decompression and replay, the
    # replay left running (asynchronous begin) while the decompressed points
    # go out -- their all-gather (RCCL on torch's stream) overlaps the replay
    # and the slice's scalar expansion on the library's stream
    job = bpperm.VerifyJob(prover.k, proofs[b:e], Vs[b:e], prover.label, ctx=prover.ctx, wait=False)
    try:
        ok = job.ok
        if ok:
            assert job.slice_bytes() <= stride and job.point_bytes() <= pstride
            ok = job.slice_points(pblk.data_ptr())  # (returns once the block is complete)
        pblocks = gather(pblk)
        if ok:
            ok = job.slice_scalars(seed, blk.data_ptr(), first=b)  # (False: the replay rejected a proof)
        blocks = gather(blk)
        torch.cuda.synchronize(dev)
        part = bytes(128)
        if ok:
            wb, we = window_ranges(_batch_windows(prover.k, len(proofs)), world)[rank]
            part = prover.verify_partial_sharded(job, b, blocks.data_ptr(), stride, pblocks.data_ptr(), pstride,
                                                 counts, wb, we)
        return ok, part
    finally:
        job.close()


def _points_per_proof(k: int) -> int:
    """Proof points of one proof in the batch MSM: V (2k + 1), A_I, A_O, S,
    T1, T3..T6, L and R (lg each)."""
    n_p = 1
    while n_p < 2 * k:
        n_p <<= 1
    return 2 * k + 1 + 8 + 2 * (n_p.bit_length() - 1)


def _batch_windows(k: int, count: int) -> int:
    """Bucket windows W of the batch MSM (msm_choose_c over its terms)."""
    import bpperm

    n_p = 1
    while n_p < 2 * k:
        n_p <<= 1
    return bpperm.msm_windows(2 * n_p + 2 + count * _points_per_proof(k))[1]


def distributed_verify(prover, proofs, Vs, rank: int, world: int, split: str = "windows", device=None,
                       seed: "bytes | None" = None) -> bool:
    """Batch-verify `proofs` (all of them, identical on every rank) with the
    MSM partitioned over the ranks (split = "windows", "windows_sharded" or
    "proofs").  seed: the batch's verifier seed, the same on every rank
    (default: drawn on rank 0 and sent to all, shared_seed)."""
    import bpperm

    if seed is None:
        seed = shared_seed(rank, device)
    if split == "windows_sharded":
        ok, part = verify_sliced(prover, proofs, Vs, rank, world, seed,
                                 lambda blk: gather_blocks(blk, world, device), device)
    elif split == "windows":
        job = bpperm.VerifyJob(prover.k, proofs, Vs, prover.label, ctx=prover.ctx)
        ok = job.ok
        if ok:
            wb, we = window_ranges(job.windows()[1], world)[rank]
            part = prover.verify_partial(job, seed, 0, wb, we)
        else:
            part = bytes(128)
        job.close()
    else:  # "proofs": no exchange before the MSM partials
        b, e = point_ranges(len(proofs), world)[rank]
        return verify_own_slice(prover, proofs[b:e], Vs[b:e], b, rank, world, device, seed)
    if part is None:  # a proof point did not decode
        ok, part = False, bytes(128)
    parts = torch_all_gather_bytes(part, device)
    # a rank that rejected a proof in its replay vetoes the batch
    flags = torch_all_gather_bytes(bytes([1 if ok else 0]), device)
    return all(f == b"\x01" for f in flags) and bpperm.partials_is_identity(parts)


def verify_own_slice(prover, proofs, Vs, first: int, rank: int, world: int, device=None,
                     seed: "bytes | None" = None) -> bool:
    """One batch verification of proofs that are already spread over the
    ranks -- config 4 as a job (BASELINE: 1024 proofs sharded across the
    GPUs): rank r holds only the proofs it proved itself, batch proofs
    [first, first + len(proofs)).  Each rank replays its own proofs and runs
    all windows of its slice's MSM, weighted as batch proofs first + p from
    the shared seed; the 128-B partials and a per-rank ok flag are
    all-gathered, and the batch verifies iff every rank's replay passed and
    the partials add up to the identity.  No proof crosses the fabric."""
    import bpperm

    if seed is None:
        seed = shared_seed(rank, device)
    job = bpperm.VerifyJob(prover.k, proofs, Vs, prover.label, ctx=prover.ctx)
    ok = job.ok
    part = prover.verify_partial(job, seed, first, 0, job.windows()[1]) if ok else None
    job.close()
    if part is None:  # a malformed proof, or a proof point that did not decode
        ok, part = False, bytes(128)
    parts = torch_all_gather_bytes(part, device)
    flags = torch_all_gather_bytes(bytes([1 if ok else 0]), device)
    return all(f == b"\x01" for f in flags) and bpperm.partials_is_identity(parts)
