#!/usr/bin/env python
"""configs[2] native runs repeated (bench.run_c3's native leg): wall time of
each rf_rifraf_batch_ref run of the 1000-read 2.6 kb cluster, to separate
run-to-run spread from a change.  usage: c3_repeat.py [runs]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import bench  # noqa: E402
import rifraf_amd.model as model  # noqa: E402
from rifraf_amd.batch import rifraf_batch  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 7
template, reads, phreds, ref = bench.c3_cluster()
params = model.RifrafParams(seed=1, batch_size=0, batch_fixed=False, do_score=True)
kw = dict(dnaseqs=reads, phreds=phreds, reference=ref)
eng = Engine(0)
rifraf_batch([kw], params=params, engine=eng, native=True)
secs = []
for _ in range(n):
    t0 = time.perf_counter()
    rifraf_batch([kw], params=params, engine=eng, native=True)
    secs.append(round(time.perf_counter() - t0, 4))
eng.close()
print(json.dumps({"native_seconds": secs, "median": sorted(secs)[len(secs) // 2]}), flush=True)
