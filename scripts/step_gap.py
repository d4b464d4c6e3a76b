"""Host time around the c4 step's two engine calls: wall time of rf_realign and
rf_score_dense against their HIP-event kernel spans (bench.py's workload)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import bench  # noqa: E402
from rifraf_amd.engine import RF_BWD, RF_FWD, Engine, pack_groups  # noqa: E402

clusters = bench.make_workload(1250, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, 0))
reads = [r for _, rs in clusters for r in rs]
nr = len(reads)
eng = Engine(0)
eng.reserve(int(sum(2 * 8 * (2 * r.bandwidth + abs(len(r) - 1500) + 1) * 1501 for r in reads) * 1.05) + (64 << 20))
for a in range(0, nr, 4096):
    eng.set_sequences(a, reads[a:a + 4096])
eng.set_templates(0, [t for t, _ in clusters])
slots = np.arange(nr, dtype=np.int32)
tpl_of = np.repeat(np.arange(len(clusters), dtype=np.int32), 50)
bws = np.array([r.bandwidth for r in reads], np.int32)
packed = pack_groups([np.arange(50 * c, 50 * c + 50, dtype=np.int32) for c in range(len(clusters))])
rec = []
for it in range(12):
    t0 = time.perf_counter()
    eng.realign(slots, slots, tpl_of, bws, RF_FWD | RF_BWD)
    t1 = time.perf_counter()
    dp = eng.last_timing()[0]
    t2 = time.perf_counter()
    eng.score_dense(packed, to_host=False)
    t3 = time.perf_counter()
    sc = eng.last_timing()[1]
    if it >= 2:
        rec.append(((t1 - t0) * 1e3, dp, (t3 - t2) * 1e3, sc, (t2 - t1) * 1e3))
r = np.array(rec)
print(json.dumps({"realign_wall_ms": r[:, 0].mean(), "dp_event_ms": r[:, 1].mean(),
                  "score_wall_ms": r[:, 2].mean(), "score_event_ms": r[:, 3].mean(),
                  "between_ms": r[:, 4].mean()}))
eng.close()
