#!/usr/bin/env python
"""End-to-end single-cluster rifraf() on one GPU for BASELINE configs[1] and
configs[2]:
  c2: sample_sequences(100, 1000; error_rate=0.01), no reference;
  c3: sample_sequences(1000, 2601; error_rate=0.01, ref_error_rate=0.1,
      ref_errors=ErrorModel(10,0,0,1,1)) with the reference (FRAME stage,
      codon-move scoring of the reference).
Default RifrafParams, seeds 1..N.  Prints one JSON line per seed with the
wall time, stage iterations, whether the consensus equals the template, and
(optional) the CPU oracle engine's time for the same call.
With a 4th argument "tp" the throughput settings are used instead of the
defaults: every read in every batch (batch_size=0, batch_fixed=false) and
the quality-score pass (do_score=true).
usage: scripts/e2e_single.py c2|c3 [SEEDS] [CPU:0/1] [tp]"""
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

from rifraf_amd import ErrorModel  # noqa: E402
from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import RifrafParams, rifraf  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
nseeds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
do_cpu = len(sys.argv) > 3 and sys.argv[3] == "1"
tp = len(sys.argv) > 4 and sys.argv[4] == "tp"
eng = Engine(0)
for seed in range(1, nseeds + 1):
    rng = np.random.default_rng(seed)
    if cfg == "c2":
        ref, t, _, reads, _, phreds, _, _ = sample_sequences(100, 1000, error_rate=0.01, rng=rng)
        kw = dict(dnaseqs=reads, phreds=phreds)
    else:
        ref, t, _, reads, _, phreds, _, _ = sample_sequences(1000, 2601, error_rate=0.01, ref_error_rate=0.1,
                                                             ref_errors=ErrorModel(10, 0, 0, 1, 1), rng=rng)
        kw = dict(dnaseqs=reads, phreds=phreds, reference=ref)
    params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True) if tp else RifrafParams()
    t0 = time.perf_counter()
    res = rifraf(params=params, engine=eng, **kw)
    gpu_s = time.perf_counter() - t0
    out = {"workload": f"{cfg}-e2e", "params": "throughput" if tp else "default", "seed": seed,
           "reads": len(reads), "template_len": len(t), "reference": cfg == "c3", "gpu_seconds": gpu_s,
           "stage_iterations": list(res.state.stage_iterations), "converged": res.state.converged,
           "consensus_equals_template": bool(np.array_equal(res.consensus, t)),
           "edit_free": int(len(res.consensus) == len(t))}
    if do_cpu:
        from oracle_engine import OracleEngine
        t0 = time.perf_counter()
        cres = rifraf(params=params, engine=OracleEngine(), **kw)
        out["cpu_baseline"] = {"seconds": time.perf_counter() - t0, "kind": "port", "cores": 1,
                               "same_consensus_as_gpu": bool(np.array_equal(cres.consensus, res.consensus)),
                               "same_score": cres.state.score == res.state.score}
    print(json.dumps(out), flush=True)
eng.close()
