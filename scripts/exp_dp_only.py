#!/usr/bin/env python
"""DP fill time alone at the c5 shape (5000 x 10 kb reads at fixed bandwidth
BW, default 18 -- the doubled width most c5 reads end at), for comparing
diagnostic builds (RIFRAF_HIP_LIB) whose bands are not valid."""
import json, os, sys
REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np
import bench
from rifraf_amd.engine import Engine, RF_BWD, RF_FWD
bw = int(sys.argv[1]) if len(sys.argv) > 1 else 18
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
t, reads = bench.make_read_shard(n, 10000, 0.03, bw, 2024, 0, n)
e = Engine(0)
e.reserve(sum(2 * bench.band_bytes(len(r), 10000, bw, pad=True) for r in reads) + (256 << 20))
e.set_sequences(0, reads)
e.set_templates(0, [t])
sl = np.arange(n, dtype=np.int32)
ms = []
for _ in range(6):
    e.realign(sl, sl, 0, bw, RF_FWD | RF_BWD)
    ms.append(e.last_timing()[0])
print(json.dumps({"bw": bw, "reads": n, "dp_ms": ms[2:], "lib": os.environ.get("RIFRAF_HIP_LIB", "default")}))
