"""CPU, world_size 2 over gloo: the multi-GPU orchestration (pair-range
scatter, delta-size all-gather, global output index, max-over-ranks timing)
that bench.py runs over RCCL on MI355X."""
from __future__ import annotations

import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import importlib.util

    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = importlib.util.spec_from_file_location(
        "shard", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "delta-compression_amd", "shard.py"))
    shard = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shard)
    sizes_in = [65536 * 2] * 10 + [262144 * 2] * 6
    ranges = shard.balanced_ranges(sizes_in, world) if rank == 0 else None
    lo, hi = shard.scatter_ranges(dist, ranges, world, rank, "cpu")
    # pretend delta sizes: 1000 + global index; the ranges are unequal
    # (byte-balanced), and SizeGather pads them internally
    counts = [b - a for a, b in shard.all_ranges(dist, ranges, world, rank, "cpu")]
    local = torch.arange(lo, hi, dtype=torch.int64) + 1000
    g = shard.SizeGather(counts, "cpu")
    allsz = g(dist, local).clone()
    off = g.global_offsets(allsz).clone()
    again = shard.gather_sizes(dist, local, world, counts)   # one-shot form
    assert again.tolist() == allsz.tolist()
    t = shard.max_over_ranks(dist, float(rank + 1), world, "cpu")
    q.put((rank, lo, hi, allsz.tolist(), off.tolist(), t))
    dist.destroy_process_group()


def test_gloo_world2_orchestration():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    # contiguous, covering, byte-balanced ranges
    (r0, lo0, hi0, s0, o0, t0), (r1, lo1, hi1, s1, o1, t1) = res
    assert lo0 == 0 and hi0 == lo1 and hi1 == 16
    assert hi0 - lo0 != hi1 - lo1   # unequal ranges, no padding by the caller
    assert s0 == s1 == [1000 + i for i in range(16)]
    assert o0 == o1 and o0[-1] == sum(s0)
    assert t0 == t1 == 2.0


def test_balanced_ranges():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "shard", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "delta-compression_amd", "shard.py"))
    shard = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shard)
    r = shard.balanced_ranges([1] * 65536, 8)
    assert r[0] == (0, 8192) and r[-1] == (57344, 65536)
    assert all(r[i][1] == r[i + 1][0] for i in range(7))
    r = shard.balanced_ranges([5, 5, 5, 5, 20], 2)
    assert r == [(0, 4), (4, 5)]
