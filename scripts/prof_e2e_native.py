#!/usr/bin/env python
"""cProfile of one process's native batched rifraf over N c4 clusters
(diagnostics: where the host time of rifraf_batch goes)."""
import cProfile, os, pstats, sys, time
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np
from rifraf_amd.batch import rifraf_batch
from rifraf_amd.engine import Engine
from rifraf_amd.model import RifrafParams
from rifraf_amd.sample import sample_sequences
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cl = []
for k in range(n):
    _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01, rng=np.random.default_rng([7, k]))
    cl.append(dict(dnaseqs=reads, phreds=phreds))
e = Engine(0)
rifraf_batch(cl[:8], params=RifrafParams(batch_size=0, batch_fixed=False, do_score=True), engine=e)   # warm
from rifraf_amd import batch as _b
for rep in range(int(os.environ.get("E2E_REPS", "0"))):   # unprofiled repetitions (warm arena)
    for k in _b.STATS:
        _b.STATS[k] = 0.0 if isinstance(_b.STATS[k], float) else 0
    t0 = time.perf_counter()
    rifraf_batch(cl, params=RifrafParams(batch_size=0, batch_fixed=False, do_score=True), engine=e)
    w = time.perf_counter() - t0
    print("rep", rep, "wall %.3f" % w, "clusters/s %.1f" % (n / w), {k: round(v, 4) for k, v in _b.STATS.items()})
for k in _b.STATS:
    _b.STATS[k] = 0.0 if isinstance(_b.STATS[k], float) else 0
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.runcall(rifraf_batch, cl, params=RifrafParams(batch_size=0, batch_fixed=False, do_score=True), engine=e)
print("wall", time.perf_counter() - t0)
from rifraf_amd import batch as _b
print("STATS", {k: round(v, 4) for k, v in _b.STATS.items()})
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
