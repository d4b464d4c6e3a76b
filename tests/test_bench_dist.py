"""bench.py's multi-rank path on CPU (gloo, world_size 2).

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


def test_aggregate_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for _, el, units in got:
        assert el == 2.0                       # slowest rank
        assert units == [30.0, 6.0, 11.0]      # whole-job units


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
