#!/usr/bin/env python3
"""RCCL rehearsal of the multi-GPU orchestration on whatever GPUs a box has:
N ranks (torch.distributed.run), rank r on cuda:(r mod device_count), backend
nccl (= RCCL).  Exercises shard.all_ranges / SizeGather (unequal counts) /
global_offsets / max_over_ranks with device tensors, plus the same all-gather
issued from a side stream behind an event (the overlap bench.py uses), and
checks every result.  On a 1-GPU box the ranks share the card."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    import importlib.util
    spec = importlib.util.spec_from_file_location("shard", os.path.join(ROOT, "delta-compression_amd", "shard.py"))
    shard = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shard)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    total = 1000 + 7 * world
    ranges = shard.balanced_ranges([1 + (i % 5) for i in range(total)], world) if rank == 0 else None
    allr = shard.all_ranges(dist, ranges, world, rank, dev)
    lo, hi = allr[rank]
    sizes = torch.arange(lo, hi, dtype=torch.int64, device=dev) * 3 + 1
    g = shard.SizeGather([b - a for a, b in allr], dev)
    got = g(dist, sizes)
    want = torch.arange(total, dtype=torch.int64, device=dev) * 3 + 1
    ok = bool(torch.equal(got, want))
    off = g.global_offsets(got)
    ok = ok and int(off[-1].item()) == int(want.sum().item())
    # side-stream all-gather behind an event, main stream moving on
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    sizes2 = sizes * 2
    ev.record()
    with torch.cuda.stream(side):
        side.wait_event(ev)
        got2 = g(dist, sizes2)
        tot2 = int(g.global_offsets(got2)[-1].item())
    ok = ok and tot2 == 2 * int(want.sum().item())
    m = shard.max_over_ranks(dist, float(rank + 1), world, dev)
    ok = ok and m == float(world)
    dist.barrier()
    if rank == 0:
        print(f'{{"rccl_rehearsal": {str(ok).lower()}, "world": {world}, "devices": {torch.cuda.device_count()}}}')
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
