#!/usr/bin/env python
"""Host time of one configs[2] (c3) rifraf_batch run outside the native
stage machine: bench's c3 cluster, two warm-up runs, then N profiled runs
under cProfile; prints batch.STATS and the top functions by cumulative and
by own time.
usage: prof_c3_host.py [N]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]

import bench  # noqa: E402
import rifraf_amd.model as model  # noqa: E402
from rifraf_amd import batch as B  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5
template, reads, phreds, ref = bench.c3_cluster()
params = model.RifrafParams(seed=1, batch_size=0, batch_fixed=False, do_score=True)
kw = dict(dnaseqs=reads, phreds=phreds, reference=ref)
eng = Engine(0)
for _ in range(2):
    B.rifraf_batch([kw], params=params, engine=eng, native=True)
ts = []
for _ in range(N):
    t0 = time.perf_counter()
    B.rifraf_batch([kw], params=params, engine=eng, native=True)
    ts.append(time.perf_counter() - t0)
print("unprofiled runs (s):", " ".join("%.4f" % t for t in ts))

pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    B.rifraf_batch([kw], params=params, engine=eng, native=True)
pr.disable()
print("batch.STATS:", getattr(B, "STATS", None))
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(40)
st.sort_stats("tottime").print_stats(30)
eng.close()
