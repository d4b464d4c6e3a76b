#!/usr/bin/env python
"""c4 bench step (realign FWD|BWD of every read + dense scoring of every
proposal) with the 1,250 clusters split over E engine contexts (own HIP
streams, own host thread), so one context's DP runs beside another's
scoring. Prints one JSON line per setting: step wall time (max over the
engines' K steps), each engine's DP / scoring kernel times, and whether the
dense totals equal the first one-engine run's (bench.parity_check's
mask: the unused p = 0 / consensus-base slots are not compared; the r05bb
record predates that mask, so its same_totals field is not meaningful).
usage: exp_c4_overlap.py K E1 [E2 ...]"""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd.engine import RF_BWD, RF_FWD, Engine, pack_groups  # noqa: E402

K = int(sys.argv[1])
settings = [int(a) for a in sys.argv[2:]] or [1, 2]
nclu, nreads, length, err, bw, _ = bench.CONFIGS["c4"]
clusters = bench.make_workload(nclu, nreads, length, err, bw, seed=bench.shard_seed(0, 0))
cells = sum(2 * bench.band_cells(len(r), len(t), r.bandwidth) for t, rs in clusters for r in rs)


class Part:
    def __init__(self, eng, cl):
        self.eng, self.cl = eng, cl
        reads = [r for _, rs in cl for r in rs]
        nr = len(reads)
        bb = sum(2 * 8 * (2 * r.bandwidth + abs(len(r) - len(t)) + 1) * (len(t) + 1) for t, rs in cl for r in rs)
        eng.reserve(int(bb * 1.05) + (64 << 20))
        for a in range(0, nr, 4096):
            eng.set_sequences(a, reads[a:a + 4096])
        eng.set_templates(0, [t for t, _ in cl])
        self.slots = np.arange(nr, dtype=np.int32)
        self.tpl = np.concatenate([[c] * len(rs) for c, (_, rs) in enumerate(cl)]).astype(np.int32)
        self.bws = np.array([r.bandwidth for r in reads], np.int32)
        groups, at = [], 0
        for _, rs in cl:
            groups.append(np.arange(at, at + len(rs), dtype=np.int32))
            at += len(rs)
        self.groups = groups
        self.packed = pack_groups(groups)
        self.dp, self.sc = [], []

    def step(self):
        self.eng.realign(self.slots, self.slots, self.tpl, self.bws, RF_FWD | RF_BWD)
        d, _, _ = self.eng.last_timing()
        self.eng.score_dense(self.packed, to_host=False)
        _, s, _ = self.eng.last_timing()
        self.dp.append(d)
        self.sc.append(s)

    def run(self, k, bar, out, i):
        bar.wait()
        t0 = time.perf_counter()
        for _ in range(k):
            self.step()
        out[i] = time.perf_counter() - t0


engs = [Engine(0) for _ in range(max(settings))]
ref = None
for rnd in range(2):
    for E in settings:
        cut = np.linspace(0, nclu, E + 1).astype(int)
        parts = [Part(engs[i], clusters[cut[i]:cut[i + 1]]) for i in range(E)]
        for p in parts:
            p.step()
            p.step()
        for p in parts:
            p.dp, p.sc = [], []
        bar = threading.Barrier(E)
        out = [0.0] * E
        th = [threading.Thread(target=p.run, args=(K, bar, out, i)) for i, p in enumerate(parts)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        dense = []
        for p in parts:
            dense += p.eng.score_dense(p.groups, rows=[len(t) + 1 for t, _ in p.cl])
        same = None
        if ref is None and E == 1:
            ref = dense
        elif ref is not None:
            same = bench.parity_check(dense, ref, [t for t, _ in clusters])["bitexact"]
        wall = max(out)
        print(json.dumps({"round": rnd, "engines": E, "steps": K, "ms_per_step": wall / K * 1e3,
                          "gcups": cells * K / wall / 1e9,
                          "dp_ms": [float(np.mean(p.dp)) for p in parts],
                          "score_ms": [float(np.mean(p.sc)) for p in parts],
                          "same_totals": same}), flush=True)
        for p in parts:
            p.eng.release_bands()
