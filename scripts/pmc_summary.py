#!/usr/bin/env python
"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, one pass each) into
profiles/pmc_<config>.json: HBM bytes per launch per hot kernel.

Corrections per MI355X_MICROARCH.md §HBM: counters are in KiB; gfx950
FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled.
k_dp = sum of the k_dpr<NP,LEAN> variants launched by one rf_realign.
usage: scripts/pmc_summary.py RUN_DIR OUT_JSON SIZE [clusters|reads]
  SIZE: clusters per rank (c4) or reads per rank (c5); bench.py matches it
  against its own run before it quotes the traffic
"""
import csv
import collections
import json
import sys


def kname(full):
    base = full.split("(")[0].replace("void ", "")
    if base.startswith("k_dpr") or base.startswith("k_dp<"):
        return "k_dp"                 # every DP class of one rf_realign
    if base.startswith("k_score"):
        return "k_score"              # k_score / k_score_lean / k_score_ws*
    return base


def per_launch(path):
    # counter rows -> {kernel: mean per dispatch}, summing the variants of one launch group
    by_disp = collections.defaultdict(float)
    name_of = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        by_disp[d] += float(r["Counter_Value"])
        name_of[d] = kname(r["Kernel_Name"])
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    # k_dp: only the DP launch group (consecutive k_dp dispatches, uploads
    # between them allowed) right before each k_score launch, i.e. the timed
    # step's realign -- not the untimed band-doubling passes of c5's setup
    group = 0.0
    for d in sorted(by_disp):
        k, v = name_of[d], by_disp[d]
        if k == "k_dp":
            group += v
        elif k == "k_score":
            tot["k_dp"] += group
            group = 0.0
        elif k not in ("k_scatter",) and not k.startswith("__amd"):
            group = 0.0
        if k != "k_dp":
            tot[k] += v
            cnt[k] += 1
    cnt["k_dp"] = cnt["k_score"]
    # per-launch means over the full-size launches only: bench --config c5
    # also launches its 16-read parity check (a fraction of a per-cent of a
    # full launch), which would otherwise pull the mean down by 1/8
    full = collections.defaultdict(list)
    group = 0.0
    for d in sorted(by_disp):
        k, v = name_of[d], by_disp[d]
        if k == "k_dp":
            group += v
            continue
        if k == "k_score":
            full["k_dp"].append(group)
        if k not in ("k_scatter",) and not k.startswith("__amd"):
            group = 0.0
        full[k].append(v)
    for k, vs in full.items():
        big = [v for v in vs if v >= 0.5 * max(vs)] if vs and max(vs) > 0 else vs
        if big:
            tot[k], cnt[k] = sum(big), len(big)
    return tot, cnt


def main():
    run, out, size = sys.argv[1], sys.argv[2], int(sys.argv[3])
    key = sys.argv[4] if len(sys.argv) > 4 else "clusters"
    f_tot, f_cnt = per_launch(f"{run}/pmc_FETCH_SIZE/p_counter_collection.csv")
    w_tot, w_cnt = per_launch(f"{run}/pmc_WRITE_SIZE/p_counter_collection.csv")
    res = {key: size, "source": run, "unit": "bytes per launch (mean over full-size launches)",
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes", "kernels": {}}
    for k in ("k_score", "k_dp"):
        if k not in f_tot:
            continue
        fetch = 2 * 1024 * f_tot[k] / max(f_cnt[k], 1)
        write = 1024 * w_tot.get(k, 0.0) / max(w_cnt.get(k, 1), 1)
        res["kernels"][k] = {"fetch_bytes": fetch, "write_bytes": write,
                             "hbm_bytes_per_launch": fetch + write}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
