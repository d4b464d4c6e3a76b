#!/usr/bin/env python
"""Experiment: overlap of the DP of one cluster chunk with the scoring of
another, using several engine contexts (own HIP streams) driven from host
threads (ctypes releases the GIL).  usage: exp_overlap.py NCTX [CLUSTERS]"""
import os, sys, threading, time, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rifraf.jl_amd"))
import numpy as np
import bench
from rifraf_amd.engine import RF_BWD, RF_FWD, Engine

nctx = int(sys.argv[1]); nclu = int(sys.argv[2]) if len(sys.argv) > 2 else 1250
clusters = bench.make_workload(nclu, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, 0))
cells = sum(2 * bench.band_cells(len(r), len(t), 9) for t, rs in clusters for r in rs)
parts = [clusters[i::nctx] for i in range(nctx)]
ctxs = []
for part in parts:
    e = Engine(0)
    reads = [r for _, rs in part for r in rs]
    e.reserve(int(sum(2 * bench.band_bytes(len(r), len(t), 9) for t, rs in part for r in rs) * 1.02) + (64 << 20))
    for a in range(0, len(reads), 4096):
        e.set_sequences(a, reads[a:a + 4096])
    e.set_templates(0, [t for t, _ in part])
    tpl_of = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(part)]).astype(np.int32)
    sl = np.arange(len(reads), dtype=np.int32)
    groups, at = [], 0
    for _, rs in part:
        groups.append(np.arange(at, at + len(rs), dtype=np.int32)); at += len(rs)
    ctxs.append((e, sl, tpl_of, groups))

def step(c):
    e, sl, tpl_of, groups = c
    e.realign(sl, sl, tpl_of, 9, RF_FWD | RF_BWD)
    e.score_dense(groups, to_host=False)

def run(steps, stagger):
    bar = threading.Barrier(nctx)
    def worker(i):
        bar.wait()
        if stagger and i:
            time.sleep(stagger * i)
        for _ in range(steps):
            step(ctxs[i])
    th = [threading.Thread(target=worker, args=(i,)) for i in range(nctx)]
    t0 = time.perf_counter()
    for t in th: t.start()
    for t in th: t.join()
    return time.perf_counter() - t0

for c in ctxs: step(c)
res = {"nctx": nctx}
for stg in (0.0, 0.004):
    dt = run(5, stg)
    res[f"stagger{stg}"] = {"ms_per_step": dt / 5 * 1e3, "gcups": cells * 5 / dt / 1e9}
print(json.dumps(res))
