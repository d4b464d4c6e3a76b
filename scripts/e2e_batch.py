#!/usr/bin/env python
"""End-to-end config-4 throughput: whole rifraf() runs (all stages, default
stage logic, batch = all 50 reads, quality scores on) over many 50 x 1.5 kb
clusters, batched on one GPU with rifraf_batch, against the same runs on the
CPU oracle engine.  Prints one JSON line.
usage: scripts/e2e_batch.py [CLUSTERS] [CPU_CLUSTERS]"""
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

from rifraf_amd.batch import STATS, rifraf_batch  # noqa: E402
from rifraf_amd.model import RifrafParams, rifraf  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402

nclu = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ncpu = int(sys.argv[2]) if len(sys.argv) > 2 else 2
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
t0 = time.perf_counter()
clusters, templates = [], []
for k in range(nclu):
    _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01, rng=np.random.default_rng([7, k]))
    clusters.append(dict(dnaseqs=reads, phreds=phreds))
    templates.append(t)
gen_s = time.perf_counter() - t0

from rifraf_amd.engine import Engine  # noqa: E402
eng = Engine(0)
t0 = time.perf_counter()
res = rifraf_batch(clusters, params=params, engine=eng)
gpu_s = time.perf_counter() - t0
ok = sum(int(np.array_equal(r.consensus, t)) for r, t in zip(res, templates))
iters = sum(sum(r.state.stage_iterations) for r in res)
cpu = None
if ncpu > 0:
    from oracle_engine import OracleEngine
    t0 = time.perf_counter()
    cres = [rifraf(params=params, engine=OracleEngine(), **kw) for kw in clusters[:ncpu]]
    cpu_s = time.perf_counter() - t0
    same = all(np.array_equal(a.consensus, b.consensus) for a, b in zip(cres, res[:ncpu]))
    cpu = {"clusters_per_s": ncpu / cpu_s, "clusters": ncpu, "seconds": cpu_s, "kind": "port",
           "cores": 1, "same_consensus_as_gpu": same}
print(json.dumps({"workload": "c4-e2e", "clusters": nclu, "reads_per_cluster": 50, "template_len": 1500,
                  "gpu_clusters_per_s": nclu / gpu_s, "gpu_seconds": gpu_s, "stage_iterations": iters,
                  "consensus_equals_template": ok,
                  "engine_calls": STATS["launches"], "engine_s": STATS["engine_s"], "setup_s": gen_s, "cpu_baseline": cpu}))
