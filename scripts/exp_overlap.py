#!/usr/bin/env python
"""Experiment: the c4 step (realign FWD|BWD + dense scoring of every
proposal) on E contexts (one HIP stream each, one host thread each), each
holding 1/E of the clusters, free-running K steps.  Whether the DP fill of
one context overlaps another's scoring on the GPU (different limiters:
the DP is issue/latency-bound at ~20 % VALU busy, the scorer LDS/VALU-bound).
Prints one JSON line per E: wall ms per step (all contexts), GCUPS.
(Round 4 also ran the fused-step prototype k_fuse here, SCORE_FWD=1; it was
removed in round 5, profiles/r04v_exp_overlap_fused.jsonl keeps the record.)"""
import json
import os
import sys
import threading
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np

import bench
from rifraf_amd.engine import RF_BWD, RF_FWD, Engine, pack_groups


def setup(clusters):
    eng = Engine(0)
    reads = [r for _, rs in clusters for r in rs]
    tpl_of = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(clusters)]).astype(np.int32)
    nr = len(reads)
    cells = sum(2 * bench.band_cells(len(r), len(t), r.bandwidth) for t, rs in clusters for r in rs)
    band_bytes = sum(2 * 8 * (2 * r.bandwidth + abs(len(r) - len(t)) + 1) * (len(t) + 1)
                     for t, rs in clusters for r in rs)
    eng.reserve(int(band_bytes * 1.05) + (64 << 20))
    for a in range(0, nr, 4096):
        eng.set_sequences(a, reads[a:a + 4096])
    eng.set_templates(0, [t for t, _ in clusters])
    slots = np.arange(nr, dtype=np.int32)
    bws = np.array([r.bandwidth for r in reads], np.int32)
    groups, at = [], 0
    for _, rs in clusters:
        groups.append(np.arange(at, at + len(rs), dtype=np.int32))
        at += len(rs)
    packed = pack_groups(groups)

    flags = RF_FWD | RF_BWD

    def step():
        eng.realign(slots, slots, tpl_of, bws, flags)
        eng.score_dense(packed, to_host=False)
    return eng, step, cells


def main():
    nclu = int(os.environ.get("NCLU", "1250"))
    steps = int(os.environ.get("STEPS", "10"))
    nclu_, nreads, length, err, bw, _ = bench.CONFIGS["c4"]
    clusters = bench.make_workload(nclu, nreads, length, err, bw, seed=bench.shard_seed(2024, 0))
    for E in [int(x) for x in os.environ.get("ENGINES", "1,2,3").split(",")]:
        parts = [clusters[k * nclu // E:(k + 1) * nclu // E] for k in range(E)]
        ctx = [setup(p) for p in parts]
        for _, st, _ in ctx:
            st()
            st()
        ts = {}

        def run(i):
            st = ctx[i][1]
            for _ in range(steps):
                st()

        th = [threading.Thread(target=run, args=(i,)) for i in range(E)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        cells = sum(c for _, _, c in ctx)
        print(json.dumps({"engines": E, "clusters": nclu, "steps": steps, "ms_per_step": wall / steps * 1e3,
                          "gcups": cells * steps / wall / 1e9}), flush=True)
        for e, _, _ in ctx:
            e.close()


if __name__ == "__main__":
    main()
