#!/usr/bin/env python
"""DP fill time alone at the c4 shape (bench.make_workload: clusters of 50
reads x 1.5 kb, bw 9; default 1250 clusters), for A/B-timing library builds
(RIFRAF_HIP_LIB), or of option settings in one process, interleaved
(argv[2], e.g. "dp_sched=0/1").  Prints one JSON line: per-call
realign(FWD|BWD) ms per setting."""
import json, os, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np
import bench
from rifraf_amd.engine import Engine, RF_BWD, RF_FWD
nclu = int(sys.argv[1]) if len(sys.argv) > 1 else 1250
clusters = bench.make_workload(nclu, 50, 1500, 0.01, 9, seed=bench.shard_seed(2024, 0))
reads = [r for _, rs in clusters for r in rs]
tpl = np.repeat(np.arange(nclu, dtype=np.int32), 50)
e = Engine(0)
e.reserve(sum(2 * bench.band_bytes(len(r), 1500, 9) for r in reads) + (256 << 20))
for a in range(0, len(reads), 4096):
    e.set_sequences(a, reads[a:a + 4096])
e.set_templates(0, [t for t, _ in clusters])
sl = np.arange(len(reads), dtype=np.int32)
bws = np.full(len(reads), 9, np.int32)
opt, vals = (sys.argv[2].split("=") if len(sys.argv) > 2 else ("dp_sched", "0"))
vals = [int(v) for v in vals.split("/")]
ms = {v: [] for v in vals}
for rnd in range(3):
    for v in vals:
        e.set_option(opt, v)
        for _ in range(5):
            e.realign(sl, sl, tpl, bws, RF_FWD | RF_BWD)
            ms[v].append(e.last_timing()[0])
print(json.dumps({"clusters": nclu, "option": opt,
                  "dp_ms": {v: [round(x, 3) for x in ms[v]] for v in vals},
                  "median": {v: float(np.median([x for k, x in enumerate(ms[v]) if k % 5])) for v in vals},
                  "lib": os.environ.get("RIFRAF_HIP_LIB", "default")}), flush=True)
