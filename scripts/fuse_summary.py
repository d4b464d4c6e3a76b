#!/usr/bin/env python
"""Summarise a fused-step A/B run (scripts/r04_fuse2.sh TAG) into
profiles/TAG_fuse.json: bench step / DP / scoring times per variant and
round, rocprofv3 kernel stats and the PMC HBM bytes per launch of the fused
step (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, KiB -> bytes).
usage: scripts/fuse_summary.py TAG"""
import collections
import csv
import glob
import json
import os
import sys

tag = sys.argv[1]
D = os.path.join("gpurun_out", tag)
out = {"tag": tag, "script": "scripts/r04_fuse2.sh", "bench": {}, "kernel_stats_ms": {}, "pmc_gb_per_launch": {}}
for f in sorted(glob.glob(os.path.join(D, "c4_*_*.json"))):
    name = os.path.basename(f)[3:-5]
    d = json.load(open(f))
    out["bench"][name] = {k: round(d[k], 3) for k in ("value", "ms_per_step", "dp_ms", "score_ms")}
    out["bench"][name]["bitexact"] = d["parity"]["bitexact"]
ks = os.path.join(D, "stats_fwd", "p_kernel_stats.csv")
if os.path.exists(ks):
    for r in csv.DictReader(open(ks)):
        out["kernel_stats_ms"][r["Name"].split("(")[0]] = {"calls": int(r["Calls"]),
                                                           "avg_ms": round(float(r["AverageNs"]) / 1e6, 3)}
for ctr, corr in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
    f = os.path.join(D, "pmc_fwd", f"pmc_{ctr}", "p_counter_collection.csv")
    if not os.path.exists(f):
        continue
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        by[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in by.items():
        if any(s in k for s in ("k_fuse", "k_reduce", "k_dpr", "k_dp<")):
            out["pmc_gb_per_launch"].setdefault(k, {})[ctr] = round(sum(v) / len(v) * 1024 * corr / 1e9, 3)
dst = os.path.join("profiles", f"{tag}_fuse.json")
json.dump(out, open(dst, "w"), indent=1)
print(dst)
print(json.dumps(out["bench"], indent=0))
