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
