"""bench.py's multi-rank path on CPU (gloo, world sizes 2 and 8).

The benchmark shards clusters over ranks with no data-path collective; the
only cross-rank step is the whole-job reduction (max time, summed units).
These tests run that reduction in two gloo processes and check the per-rank
sharding and the in-band cell count the metric is built on.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        el, units = bench.aggregate(1.0 + rank, [10.0 * (rank + 1), 3.0, 5.0 + rank])
        q.put((rank, el, units))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_aggregate_ranks(world):
    """Max-over-ranks time and summed units, at 2 ranks and at the 8 of a
    node (the only world size north_star scores)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, el, units in got:
        assert el == float(world)              # slowest rank
        assert units == [10.0 * world * (world + 1) / 2, 3.0 * world,
                         5.0 * world + world * (world - 1) / 2]   # whole-job units


def _bench(args, env=None, timeout=300):
    import json
    import subprocess
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=e, cwd=REPO,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, [json.loads(ln) for ln in lines]


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launches_ranks(world):
    """`bench.py --gpus N` with no launcher starts N ranks itself: one JSON
    line (rank 0) whose reduction covers every rank's shard (N = 8: the
    driver's scaling run on one node, rehearsed with gloo)."""
    p, lines = _bench(["--gpus", str(world), "--backend", "gloo", "--config", "c4", "--clusters", "2",
                       "--e2e-clusters", "3", "--no-cpu", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1
    # stdout carries the JSON line only (gloo's connection report goes to stderr)
    assert [ln for ln in p.stdout.splitlines() if ln.strip()] == [p.stdout.strip()]
    out = lines[0]
    assert out["ranks"] == world and out["n_gpus"] == world
    assert out["reads_all_ranks"] == world * 2 * 50
    cells = sum(2 * bench.band_cells(len(r), len(t), r.bandwidth)
                for rank in range(world)
                for t, rs in bench.make_workload(2, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, rank))
                for r in rs)
    assert out["cells_per_step_all_ranks"] == cells
    # the per-rank spread of the static shards (bench `rank_balance` measures their time)
    per_rank = [sum(2 * bench.band_cells(len(r), len(t), r.bandwidth)
                    for t, rs in bench.make_workload(2, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, rank))
                    for r in rs) for rank in range(world)]
    assert out["rank_cells_min_max"] == [min(per_rank), max(per_rank)]
    # the e2e field's hand-out (pmap's dynamic queue, scripts/rifraf.jl:190): one
    # global list staged by the ranks, every cluster taken exactly once over all
    # ranks and read back identical to one process's simulation of it
    h = out["e2e_hand_out"]
    assert h["clusters"] == world * 3 and h["exactly_once"] and h["identical_to_one_process"]
    assert sum(h["per_rank"]) == world * 3


def test_bench_rejects_world_mismatch():
    """Under an external launcher the world size must equal --gpus."""
    p, lines = _bench(["--gpus", "2", "--dry-run", "--config", "c4", "--clusters", "1"],
                      env={"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and not lines
    assert "WORLD_SIZE=1" in p.stderr


def test_shards_are_independent():
    a = bench.make_workload(2, 3, 60, 0.01, 9, seed=bench.shard_seed(7, 0))
    b = bench.make_workload(2, 3, 60, 0.01, 9, seed=bench.shard_seed(7, 1))
    a2 = bench.make_workload(2, 3, 60, 0.01, 9, seed=bench.shard_seed(7, 0))
    assert not np.array_equal(a[0][0], b[0][0])
    for (t1, r1), (t2, r2) in zip(a, a2):        # deterministic per rank
        assert np.array_equal(t1, t2)
        assert all(np.array_equal(x.seq, y.seq) for x, y in zip(r1, r2))


@pytest.mark.parametrize("n,m,bw", [(10, 10, 3), (12, 7, 2), (5, 20, 9), (1500, 1487, 9), (1, 1, 1)])
def test_band_cells_matches_geometry(n, m, bw):
    """band_cells = number of in-band cells (bandedarrays.jl:133-137)."""
    nrows, ncols = n + 1, m + 1
    h_off, v_off = max(ncols - nrows, 0), max(nrows - ncols, 0)
    count = sum(1 for i in range(nrows) for j in range(ncols) if j - h_off - bw <= i <= j + v_off + bw)
    assert bench.band_cells(n, m, bw) == count
