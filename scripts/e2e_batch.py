#!/usr/bin/env python
"""End-to-end config-4 throughput: whole rifraf() runs (all stages, default
stage logic, batch = all 50 reads, quality scores on) over many 50 x 1.5 kb
clusters, batched on one GPU with rifraf_batch, against the same runs on the
CPU oracle engine.  Prints one JSON line.
usage: scripts/e2e_batch.py [CLUSTERS] [CPU_CLUSTERS] [PROCS] [native|hub]
PROCS > 1: that many worker processes, each with its own engine context on
GPU 0 and a contiguous share of the clusters (the reference's pmap workers,
scripts/rifraf.jl:190); the host stage machine is the per-process limit."""
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

nproc = int(sys.argv[3]) if len(sys.argv) > 3 else 1
native = (sys.argv[4] != "hub") if len(sys.argv) > 4 else None


def _shard(args):
    lo, hi = args
    from rifraf_amd.batch import STATS as st
    from rifraf_amd.engine import Engine
    e = Engine(0)
    out = rifraf_batch(clusters[lo:hi], params=params, engine=e, native=native)
    e.close()
    return [(r.consensus, sum(r.state.stage_iterations)) for r in out], st["launches"], st["engine_s"]


if nproc <= 1:
    from rifraf_amd.engine import Engine  # noqa: E402
    eng = Engine(0)
    t0 = time.perf_counter()
    res = rifraf_batch(clusters, params=params, engine=eng, native=native)
    gpu_s = time.perf_counter() - t0
    cons = [r.consensus for r in res]
    iters = sum(sum(r.state.stage_iterations) for r in res)
else:
    import multiprocessing as mp
    bounds = [k * nclu // nproc for k in range(nproc + 1)]
    with mp.get_context("fork").Pool(nproc) as pool:      # fork before any HIP call
        t0 = time.perf_counter()
        parts = pool.map(_shard, list(zip(bounds[:-1], bounds[1:])))
        gpu_s = time.perf_counter() - t0
    cons = [c for part, _, _ in parts for c, _ in part]
    iters = sum(i for part, _, _ in parts for _, i in part)
    STATS["launches"] = sum(p[1] for p in parts)
    STATS["engine_s"] = sum(p[2] for p in parts)
ok = sum(int(np.array_equal(c, t)) for c, t in zip(cons, templates))
cpu = None
if ncpu > 0:
    from oracle_engine import OracleEngine
    t0 = time.perf_counter()
    cres = [rifraf(params=params, engine=OracleEngine(), **kw) for kw in clusters[:ncpu]]
    cpu_s = time.perf_counter() - t0
    same = all(np.array_equal(a.consensus, b) for a, b in zip(cres, cons[:ncpu]))
    cpu = {"clusters_per_s": ncpu / cpu_s, "clusters": ncpu, "seconds": cpu_s, "kind": "port",
           "cores": 1, "same_consensus_as_gpu": same}
print(json.dumps({"workload": "c4-e2e", "clusters": nclu, "procs": nproc, "reads_per_cluster": 50, "template_len": 1500,
                  "gpu_clusters_per_s": nclu / gpu_s, "gpu_seconds": gpu_s, "stage_iterations": iters,
                  "consensus_equals_template": ok,
                  "engine_calls": STATS["launches"], "engine_s": STATS["engine_s"], "native_s": STATS["native_s"],
                  "score_phase_s": STATS["score_phase_s"], "setup_native_s": STATS["setup_native_s"], "upload_s": STATS["upload_s"], "driver": "hub" if native is False else "native-if-eligible",
                  "setup_s": gen_s, "cpu_baseline": cpu}))
