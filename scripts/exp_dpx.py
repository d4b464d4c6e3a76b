#!/usr/bin/env python
"""Latency-bound DP fills at the configs[2] shape, for A/B-timing library
builds (RIFRAF_HIP_LIB): the reference's codon DP alone (one k_dpx<true, true>
task, 2,622 x 2,601, bw 9), the 1,000 reads alone (bw 18, latency mode:
k_dpx<false, false>; and dp_lat 0: the throughput classes), and the
edit_distance band (bw = ceil(min(m, n) / 2), k_dp<DPW_NT>).  One JSON line:
median kernel ms per call (HIP events) and ns per anti-diagonal."""
import json
import math
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rifraf.jl_amd")]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from rifraf_amd import ErrorModel, RifrafSequence, Scores  # noqa: E402
from rifraf_amd.engine import RF_FWD, RF_SKEW, Engine, RifrafError  # noqa: E402

template, reads, phreds, ref = bench.c3_cluster()
m = len(template)
ref_scores = Scores.from_errors(ErrorModel(10.0, 0.1, 0.1, 1.0, 1.0))
rseq = RifrafSequence(ref, np.full(len(ref), math.log10(0.1)), 9, ref_scores)
seq_scores = Scores.from_errors(ErrorModel(1.0, 2.0, 2.0, 0.0, 0.0))
rs = [RifrafSequence(r, -p / 10.0, 18, seq_scores) for r, p in zip(reads, phreds)]
ebw = int(math.ceil(min(m, len(ref)) * 0.5))
eseq = RifrafSequence(ref, np.full(len(ref), -1.0), ebw, Scores.from_errors(ErrorModel(1.0, 1.0, 1.0)))

e = Engine(0)
e.set_sequences(0, rs + [rseq, eseq])
e.set_templates(0, [template])
nr = len(rs)


def timed(slots, seqs, bws, flags, reps=6):
    ms = []
    for _ in range(reps):
        try:
            e.realign(np.asarray(slots, np.int32), np.asarray(seqs, np.int32), 0, np.asarray(bws, np.int32), flags)
        except RifrafError:   # diagnostic builds compute wrong bands
            if "librifraf_hip" in out["lib"]:
                raise
        ms.append(e.last_timing()[0])
    return float(np.median(ms[1:]))


out = {"lib": os.environ.get("RIFRAF_HIP_LIB", "default")}
K_ref = (2 * 9 + abs(len(ref) - m) + 1) + 2 * m
out["ref_ms"] = timed([nr], [nr], [9], RF_FWD)
out["ref_skew_ms"] = timed([nr], [nr], [9], RF_FWD | RF_SKEW)
out["ref_ns_per_step"] = out["ref_ms"] * 1e6 / K_ref
out["reads_lat_ms"] = timed(range(nr), range(nr), [18] * nr, RF_FWD)
e.set_option("dp_lat", 0)
out["reads_thr_ms"] = timed(range(nr), range(nr), [18] * nr, RF_FWD)
e.set_option("dp_lat", 2048)
out["reads_plus_ref_ms"] = timed(list(range(nr)) + [nr], list(range(nr)) + [nr], [18] * nr + [9], RF_FWD)
out["edit_ms"] = timed([nr + 1], [nr + 1], [ebw], RF_FWD | RF_SKEW, reps=3)
e.close()
print(json.dumps(out), flush=True)
