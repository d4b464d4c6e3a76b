#!/usr/bin/env python
"""edit_distance's band at configs[2]'s shape (2,622 x 2,601, skew, bw =
ceil(min / 2): H = 2,623) filled alone: per-call ms (HIP events) of
rf_realign with RF_OPT_DP_MC 1 (k_dpm) and 0 (k_dp; k_dpw before round 6), for the library named
by RIFRAF_HIP_LIB.  With library names as arguments it runs itself once per
library (child processes) and prints one JSON line each.
usage: exp_dpm.py [lib.so ...]"""
import json
import math
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:
    for lib in sys.argv[1:]:
        env = dict(os.environ, RIFRAF_HIP_LIB=os.path.join(REPO, "rifraf.jl_amd", lib))
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                           timeout=300)
        print(r.stdout.strip() or r.stderr[-800:], flush=True)
        if r.returncode:
            sys.exit(r.returncode)
    sys.exit(0)
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd import ErrorModel, RifrafSequence, Scores  # noqa: E402
from rifraf_amd.engine import RF_FWD, RF_SKEW, Engine  # noqa: E402

template, reads, phreds, ref = bench.c3_cluster()
bw = int(math.ceil(min(len(template), len(ref)) * 0.5))
r = RifrafSequence(ref, np.full(len(ref), -1.0), bw, Scores.from_errors(ErrorModel(1.0, 1.0, 1.0)))
e = Engine(0)
e.set_sequences(0, [r])
e.set_templates(0, [template])
out = {"lib": os.path.basename(os.environ.get("RIFRAF_HIP_LIB", "librifraf_hip.so")),
       "H": 2 * bw + abs(len(ref) - len(template)) + 1}
for mc in (1, 0):
    e.set_option("dp_mc", mc)
    ms, sc = [], None
    for _ in range(6):
        s = e.realign([0], [0], 0, [bw], RF_FWD | RF_SKEW)
        ms.append(round(e.last_timing()[0], 3))
        sc = float(s[0]) if sc is None else sc
        assert float(s[0]) == sc
    out[f"mc{mc}_ms"] = ms
    out[f"mc{mc}_score"] = sc
out["same_score"] = out["mc1_score"] == out["mc0_score"]
e.close()
print(json.dumps(out), flush=True)
