"""Host-side profile of whole rifraf() runs (config-4 shape: 50 x 1.5 kb,
throughput settings) on one engine, one after another, under cProfile.
usage: python scripts/prof_single.py [CLUSTERS]  -> gpurun_out/single.prof + top list"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

from rifraf_amd.engine import Engine  # noqa: E402
from rifraf_amd.model import RifrafParams, rifraf  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
params = RifrafParams(batch_size=0, batch_fixed=False, do_score=True)
clusters = []
for k in range(n):
    _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01, rng=np.random.default_rng([7, k]))
    clusters.append((t, reads, phreds))
eng = Engine(0)
rifraf(clusters[0][1], clusters[0][2], params=params, engine=eng)      # warm-up (uploads, plans)
prof = cProfile.Profile()
t0 = time.perf_counter()
prof.enable()
ok = 0
for t, reads, phreds in clusters:
    r = rifraf(reads, phreds, params=params, engine=eng)
    ok += int(np.array_equal(r.consensus, t))
prof.disable()
dt = time.perf_counter() - t0
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
prof.dump_stats(os.path.join(REPO, "gpurun_out", "single.prof"))
print(f"{n} clusters in {dt:.2f} s ({n / dt:.1f} clusters/s), consensus == template: {ok}")
pstats.Stats(prof).sort_stats("tottime").print_stats(35)
