#!/usr/bin/env python
"""Where a rank's e2e pass spends its time, unpinned and pinned to 2 cores
(bench.py's e2e field at N = 1: 512 c4-shape clusters, all reads, QVs,
ClusterQueue waves taken by E engine threads): per setting, alternating
rounds of (unpinned, pinned) passes, each pass's wall time and its phase
timeline (batch.TIMELINE: setup, upload, prep, native, results, qv per
engine thread).

usage: e2e_phases.py [N] [E/W[/X[/B[/S]]] ...]
  (engines, wave, init_exclusive 0, sync_block 0 (2: auto), setup_exclusive 1)"""
import json
import os
import resource
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd import batch as B  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import RifrafParams  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
settings = [tuple(int(x) for x in a.replace("/", ",").split(",")) for a in sys.argv[2:]] or [(2, 256)]
settings = [st + (0, 0, 1)[len(st) - 2:] for st in settings]
data = bench.E2EClusters(2024, n, 0, 1)
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
engs = [Engine(0) for _ in range(max(st[0] for st in settings))]
for e in engs:
    B.rifraf_batch([data.get(k) for k in range(4)], params=params, engine=e)
allowed = sorted(os.sched_getaffinity(0))
pin = allowed[:2]


def one(ne, wave, excl, sx):
    q = B.ClusterQueue(n, wave)
    B.TIMELINE = []
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    B.rifraf_batch_queue(data.get, q, params=params, engines=engs[:ne], init_exclusive=bool(excl),
                         setup_exclusive=bool(sx))
    wall = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    tl = [(th, ph, round(a - t0, 4), round(b - t0, 4), round(c, 4)) for th, ph, a, b, c in B.TIMELINE]
    B.TIMELINE = None
    phases = {"process_cpu_s": round(ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, 4)}
    for _, ph, a, b, c in tl:
        phases[ph] = round(phases.get(ph, 0.0) + b - a, 4)
        phases[ph + "_cpu"] = round(phases.get(ph + "_cpu", 0.0) + c, 4)
    return wall, phases, tl


for ne, wave, excl, blk, sx in settings:
    for e in engs:
        e.set_option("sync_block", blk)
    one(ne, wave, excl, sx)      # arenas sized
    rows = {"unpinned": [], "pinned": []}
    for rnd in range(3):
        rows["unpinned"].append(one(ne, wave, excl, sx))
        saved = bench.pin_threads(pin)
        try:
            rows["pinned"].append(one(ne, wave, excl, sx))
        finally:
            bench.unpin_threads(saved)
    med = {k: sorted(v, key=lambda x: x[0])[1] for k, v in rows.items()}
    print(json.dumps({"engines": ne, "wave": wave, "init_exclusive": excl, "sync_block": blk, "setup_exclusive": sx,
                      "walls": {k: [round(x[0], 4) for x in v] for k, v in rows.items()},
                      "ratio_median": round(med["unpinned"][0] / med["pinned"][0], 3),
                      "phases_median": {k: v[1] for k, v in med.items()},
                      "timeline_median": {k: v[2] for k, v in med.items()}}), flush=True)
for e in engs:
    e.close()
