#!/usr/bin/env python
"""Band row stride A/B at the c4 shape (round 6, profiles/r08d): for each
library named (built at commit db2b22a with RIFRAF_BAND_ODD = 1 / 0: kappa
rows of ceil(H/2) | 1 or ceil(H/2) doubles; the even layout and its NP = 1
stride classes were not kept), the DP fill alone (realign FWD|BWD, HIP-event ms, 3 x 5 calls)
and, for the first 64 reads, the scores and the downloaded A / B bands
(column-major, layout independent) hashed, so both layouts must agree.
usage: exp_band_stride.py nclusters lib.so [lib.so ...]"""
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2:
    for lib in sys.argv[2:]:
        env = dict(os.environ, RIFRAF_HIP_LIB=os.path.join(REPO, "rifraf.jl_amd", lib))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), sys.argv[1]], env=env, capture_output=True,
                           text=True, timeout=300)
        print(r.stdout.strip() or r.stderr[-800:], flush=True)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd.engine import RF_BAND_A, RF_BAND_B, RF_BWD, RF_FWD, Engine  # noqa: E402

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
ms = []
sc = None
for _ in range(15):
    out = e.realign(sl, sl, tpl, bws, RF_FWD | RF_BWD)
    ms.append(e.last_timing()[0])
    sc = out if sc is None else sc
h = hashlib.sha256(np.ascontiguousarray(sc).tobytes())
for k in range(64):
    for which in (RF_BAND_A, RF_BAND_B):
        h.update(np.ascontiguousarray(e.download_band(k, which).data).tobytes())
print(json.dumps({"lib": os.path.basename(os.environ.get("RIFRAF_HIP_LIB", "librifraf_hip.so")), "clusters": nclu,
                  "dp_ms": [round(x, 3) for x in ms], "median": float(np.median(ms[1:])),
                  "device_bytes": e.device_bytes(), "hash": h.hexdigest()[:16]}), flush=True)
