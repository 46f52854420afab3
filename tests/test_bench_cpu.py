"""CPU: bench.py's launcher and its multi-rank orchestration (VERDICT r1
items 3/7).  `bench.py --gpus N` with no WORLD_SIZE starts N ranks itself
under torch.distributed.run; --dry-run runs them over gloo with no GPU call;
A/B switches in the environment make bench.py refuse to measure."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("DG_") and k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **kw)
    return env


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_launches_n_ranks(gpus):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(gpus), "--dry-run"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one line
    d = lines[0]
    assert d["n_gpus"] == gpus
    assert d["index_ok"] is True
    rng = d["ranges"]
    assert rng[0][0] == 0 and all(rng[i][1] == rng[i + 1][0] for i in range(gpus - 1))
    assert len({b - a for a, b in rng}) > 1   # the unequal-range case is exercised
    # value counts the all-reduced sum of every rank's bytes
    assert d["bytes_job"] == d["bytes_expected"]
    assert d["bytes_rank0_x_world"] != d["bytes_expected"]


def test_bench_rejects_world_mismatch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_bench_refuses_ab_switches():
    r = subprocess.run([sys.executable, BENCH, "--steps", "1", "--warmup", "0"],
                       env=_env(DG_SERIAL_CRC="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "refusing" in (r.stderr + r.stdout)
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_compact_line_fits_driver_tail():
    """The printed line stays <= 4 KB with every config under `also`
    (a 20 KB line overflowed the driver's stdout tail)."""
    sys.path.insert(0, ROOT)
    import bench
    full = json.load(open(os.path.join(ROOT, "profiles", "r03_bench_default_final.json")))
    also = full.pop("also")
    names = [n for n in bench.CONFIGS if n != "c2"]
    also = {n: dict(also[n if n in also else "c3"]) for n in names}
    txt = bench.compact_line(full, also, "gpurun_out/bench_full.json")
    assert len(txt) <= bench.LINE_MAX
    d = json.loads(txt)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "cpu_baseline"):
        assert k in d
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"]
    assert d["cpu_baseline"]["cores"] and d["cpu_baseline"]["kind"] == "reference"
    assert set(d["also"]) == set(names)
    assert all("value" in e and "frac" in e for e in d["also"].values())


@pytest.mark.parametrize("steps,warmup", [(1, 0), (2, 1), (3, 5), (5, 2), (100, 20), (101, 0)])
def test_timing_ring_holds_only_timed_steps(steps, warmup):
    """bench.py records the kernel events on every `every`-th step after
    set_timing (the first, then every k-th, warmup steps included); the ring
    of `slots` recorded runs must lie inside the K timed steps and not be
    empty (plain simulation of dg_*_plan_set_timing_every)."""
    sys.path.insert(0, ROOT)
    try:
        import bench
    finally:
        sys.path.remove(ROOT)
    every, slots = bench.timing_ring(steps)
    recorded = [i for i in range(warmup + steps) if i % every == 0]
    ring = recorded[-slots:]
    assert ring and all(i >= warmup for i in ring), (every, slots, ring)
    assert every <= bench.TIMING_EVERY
