#!/usr/bin/env python
"""bench.py's e2e workload (512 c4-shape clusters, all reads, QVs) through
rifraf_batch with the process pinned to K host cores (every thread, in
place) and E engines (contexts on their own host threads), optionally with
blocking-sync host waits (B = 1: RF_OPT_SYNC_BLOCK), waves of W clusters
taken from a shared queue and X = 1: at most one engine in its native stage
machine at a time (rifraf_batch(init_exclusive=True), a two-stage pipeline):
wall time and the stage split (batch.STATS) per setting, so the host work
that does not fit a rank's 2-core share at 8 ranks shows up.
usage: e2e_pinned.py [N] [K,E[,B[,W[,X]]] ...]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd import batch as B  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import RifrafParams  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
settings = [tuple(int(x) for x in a.split(",")) for a in sys.argv[2:]] or [(16, 1), (2, 1), (2, 2), (16, 2)]
settings = [st + (0, 1024, 0)[len(st) - 2:] for st in settings]
cl = []
for k in range(n):
    _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01,
                                                        rng=np.random.default_rng([2024, 77, 0, k]))
    cl.append(dict(dnaseqs=reads, phreds=phreds))
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
engs = [Engine(0) for _ in range(max(st[1] for st in settings))]
for e in engs:
    B.rifraf_batch(cl[:4], params=params, engine=e)
B.rifraf_batch(cl, params=params, engines=engs)       # arenas sized
allowed = sorted(os.sched_getaffinity(0))
ref = None
for cores, ne, blk, wv, excl in settings:
    for e in engs:
        e.set_option("sync_block", blk)
    saved = bench.pin_threads(allowed[:cores]) if cores < len(allowed) else None
    try:
        for rep in range(2):
            for k in B.STATS:
                B.STATS[k] = 0.0 if isinstance(B.STATS[k], float) else 0
            t0 = time.perf_counter()
            res = B.rifraf_batch(cl, params=params, engines=engs[:ne], wave=wv, init_exclusive=bool(excl))
            w = time.perf_counter() - t0
        cons = [r.consensus.tobytes() for r in res]
        ref = ref or cons
        print(json.dumps({"cores": cores, "engines": ne, "sync_block": blk, "wave": wv, "init_exclusive": excl,
                          "same_consensus": cons == ref, "wall_s": round(w, 4), "clusters_per_s": round(n / w, 1),
                          "stats": {k: round(v, 4) for k, v in B.STATS.items()}}), flush=True)
    finally:
        if saved:
            bench.unpin_threads(saved)
for e in engs:
    e.close()
