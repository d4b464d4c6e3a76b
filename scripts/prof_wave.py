#!/usr/bin/env python
"""cProfile of one native e2e wave (256 c4-shape clusters, all reads, QVs)
on one engine after warm-up: where the host time of a wave goes.
usage: prof_wave.py [clusters] [lines]"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]

import bench  # noqa: E402
from rifraf_amd import batch as B  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import RifrafParams  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
lines = int(sys.argv[2]) if len(sys.argv) > 2 else 45
data = bench.E2EClusters(2024, n, 0, 1)
cl = [data.get(k) for k in range(n)]
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
e = Engine(0)
B.rifraf_batch(cl, params=params, engine=e, wave=n)
B.rifraf_batch(cl, params=params, engine=e, wave=n)
B.TIMELINE = []
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.runcall(B.rifraf_batch, cl, params=params, engine=e, wave=n)
wall = time.perf_counter() - t0
print(f"wall {wall:.4f} s for {n} clusters")
for th, ph, a, b, *_ in B.TIMELINE:
    print(f"  {ph:8s} {b - a:.4f}")
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(lines)
    print(s.getvalue())
e.close()
