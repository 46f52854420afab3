"""Multi-GPU orchestration of a pair batch (one process per GPU).

The path shards trivially: pairs are independent, so each rank encodes a
contiguous range of pair indices with no data-path collective.  The only
collectives (RCCL over xGMI on MI355X; gloo in the CPU tests) are:

* ``scatter_ranges`` — rank 0 decides the per-rank [lo, hi) index ranges,
  balanced by input bytes, and broadcasts them (world x 16 B);
* ``gather_sizes``   — an all-gather of per-pair delta sizes, from which every
  rank derives the global packed-output index (8 B per pair);
* ``max_over_ranks`` — max-reduce of the timed region.

No payload byte crosses the interconnect.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def balanced_ranges(pair_bytes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous ranges with near-equal sum(|R|+|V|) per rank."""
    n = len(pair_bytes)
    total = sum(pair_bytes)
    out, lo, acc = [], 0, 0
    for r in range(world):
        if r == world - 1:
            out.append((lo, n))
            break
        target = total * (r + 1) / world
        hi = lo
        while hi < n and acc + pair_bytes[hi] <= target:
            acc += pair_bytes[hi]
            hi += 1
        out.append((lo, hi))
        lo = hi
    return out


def scatter_ranges(dist, ranges: Sequence[Tuple[int, int]] | None, world: int, rank: int,
                   device) -> Tuple[int, int]:
    """Rank 0's ranges to every rank; returns this rank's (lo, hi)."""
    import torch
    t = torch.zeros((world, 2), dtype=torch.int64, device=device)
    if rank == 0:
        t.copy_(torch.tensor(ranges, dtype=torch.int64))
    if world > 1:
        dist.broadcast(t, src=0)
    lo, hi = t[rank].tolist()
    return int(lo), int(hi)


def gather_sizes(dist, sizes, world: int):
    """All-gather equal-length per-rank size vectors -> (world*n,) tensor."""
    import torch
    if world == 1:
        return sizes.clone()
    out = torch.empty(world * sizes.numel(), dtype=sizes.dtype, device=sizes.device)
    dist.all_gather_into_tensor(out, sizes)
    return out


def global_offsets(all_sizes):
    """Exclusive prefix sum: where each pair's delta lands in a global arena."""
    import torch
    off = torch.zeros(all_sizes.numel() + 1, dtype=torch.int64, device=all_sizes.device)
    off[1:] = torch.cumsum(all_sizes, 0)
    return off


def max_over_ranks(dist, value: float, world: int, device) -> float:
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
