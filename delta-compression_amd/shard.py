"""Multi-GPU orchestration of a pair batch (one process per GPU).

The path shards trivially: pairs are independent, so each rank encodes a
contiguous range of pair indices with no data-path collective.  The only
collectives (RCCL over xGMI on MI355X; gloo in the CPU tests) are:

* ``scatter_ranges`` — rank 0 decides the per-rank [lo, hi) index ranges,
  balanced by input bytes, and broadcasts them (world x 16 B);
* ``SizeGather``     — an all-gather of per-pair delta sizes (8 B per pair,
  ranges of unequal length padded internally), from which every rank derives
  the global packed-output index with ``global_offsets``;
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
    lo_hi = all_ranges(dist, ranges, world, rank, device)
    return lo_hi[rank]


def all_ranges(dist, ranges: Sequence[Tuple[int, int]] | None, world: int, rank: int,
               device) -> List[Tuple[int, int]]:
    """Rank 0's ranges, broadcast: every rank learns every rank's (lo, hi)."""
    import torch
    t = torch.zeros((world, 2), dtype=torch.int64, device=device)
    if rank == 0:
        t.copy_(torch.tensor(ranges, dtype=torch.int64))
    if world > 1:
        dist.broadcast(t, src=0)
    return [(int(a), int(b)) for a, b in t.tolist()]


class SizeGather:
    """All-gather of per-rank delta-size vectors of possibly unequal length.

    ``counts[r]`` is rank r's number of pairs (known to every rank from the
    broadcast ranges).  The collective moves fixed-size blocks of
    ``max(counts)`` entries, so each rank's vector is padded into a
    preallocated block and the gathered blocks are compacted back to the
    global pair order with a precomputed index.  All buffers are allocated
    once; a call does one copy, one all-gather and one gather."""

    def __init__(self, counts: Sequence[int], device, dtype=None):
        import torch
        self.counts = [int(c) for c in counts]
        self.world = len(self.counts)
        self.nmax = max(self.counts) if self.counts else 0
        dtype = dtype or torch.int64
        self.block = torch.zeros(self.nmax, dtype=dtype, device=device)
        self.padded = torch.empty(self.world * self.nmax, dtype=dtype, device=device)
        idx = [r * self.nmax + i for r, c in enumerate(self.counts) for i in range(c)]
        self.index = torch.tensor(idx, dtype=torch.int64, device=device)
        self.equal = all(c == self.nmax for c in self.counts)
        self.out = torch.empty(len(idx), dtype=dtype, device=device)
        self.offsets = torch.zeros(len(idx) + 1, dtype=torch.int64, device=device)

    def __call__(self, dist, sizes):
        """-> (sum(counts),) sizes in global pair order (a view of ``self.out``)."""
        import torch
        n = sizes.numel()
        if self.world == 1:
            self.out.copy_(sizes)
            return self.out
        if self.equal:
            dist.all_gather_into_tensor(self.out, sizes.contiguous())
            return self.out
        self.block[:n].copy_(sizes)
        dist.all_gather_into_tensor(self.padded, self.block)
        torch.index_select(self.padded, 0, self.index, out=self.out)
        return self.out

    def global_offsets(self, all_sizes):
        """Exclusive prefix sum into the preallocated offsets (n+1 entries)."""
        import torch
        torch.cumsum(all_sizes, 0, out=self.offsets[1:])
        return self.offsets


def gather_sizes(dist, sizes, world: int, counts: Sequence[int] | None = None):
    """One-shot form of SizeGather: counts default to equal lengths."""
    counts = list(counts) if counts is not None else [sizes.numel()] * world
    return SizeGather(counts, sizes.device, sizes.dtype)(dist, sizes).clone()


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


def sum_over_ranks(dist, value: int, world: int, device) -> int:
    """The job's total of a per-rank count (bytes processed): ranks hold
    byte-balanced but unequal pair ranges, so rank 0's count times the world
    size is not the total."""
    import torch
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())
