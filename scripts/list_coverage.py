#!/usr/bin/env python
"""How much of the dense scoring pass would a list-sized scorer skip?
(VERDICT r03 Next 8.)  Runs bench.py's e2e clusters (c4 shape, all reads,
QVs) through the Python stage machine on the oracle engine (CPU) and records
every proposal list scored by rf_score (get_candidates: INIT alignment
proposals): its size against the dense pass (8m + 4 proposals), and the
fraction of the k_score_ws work units (256-column windows, and 64-column
windows) that hold at least one proposal -- the column windows a list-sized
scorer would still have to stage and run.  usage: list_coverage.py [N]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

from oracle_engine import OracleEngine  # noqa: E402
from rifraf_amd.model import RifrafParams, rifraf  # noqa: E402
from rifraf_amd.proposals import to_arrays  # noqa: E402
from rifraf_amd.sample import sample_sequences  # noqa: E402


class Rec(OracleEngine):
    def __init__(self):
        super().__init__()
        self.calls = []

    def score(self, groups, per_seq=False):
        for bslots, ref, props in groups:
            k, p, b = props if isinstance(props, tuple) else to_arrays(props)
            m = len(self.tpls[0][0])
            cols = np.unique(np.asarray(p))
            self.calls.append({"P": len(k), "dense": 8 * m + 4, "m": m,
                               "win256": len(np.unique(cols // 256)) / ((m + 256) // 256),
                               "win64": len(np.unique(cols // 64)) / ((m + 64) // 64)})
        return super().score(groups, per_seq)


n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
rows = []
for k in range(n):
    _, t, _, reads, _, phreds, _, _ = sample_sequences(50, 1500, error_rate=0.01,
                                                        rng=np.random.default_rng([2024, 77, 0, k]))
    e = Rec()
    rifraf(reads, phreds, params=RifrafParams(batch_size=0, batch_fixed=False, do_score=True), engine=e)
    rows += e.calls
P = np.array([r["P"] for r in rows])
D = np.array([r["dense"] for r in rows])
out = {"clusters": n, "list_calls": len(rows), "proposals_per_call_mean": float(P.mean()),
       "proposals_over_dense_mean": float((P / D).mean()),
       "windows256_touched_mean": float(np.mean([r["win256"] for r in rows])),
       "windows64_touched_mean": float(np.mean([r["win64"] for r in rows])),
       "note": "a list-sized scorer still stages and scores every column window that holds a proposal"}
print(json.dumps(out))
