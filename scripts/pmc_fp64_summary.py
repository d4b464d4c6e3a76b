#!/usr/bin/env python
"""Summarise the FP64 PMC passes (scripts/pmc_fp64.sh; round 3: pmc_r03.sh)
into profiles/.

  pmc_fp64.json   FP64 VALU instruction counts (SQ_INSTS_VALU_{ADD,MUL,FMA,
                  TRANS}_F64) per kernel at c4 and c5, the issued FP64 lane-op
                  rate of each launch against the FP64 vector peak, and the DP
                  fill's FP64 lane-ops per in-band cell (bench.py scales that
                  ratio by its own cells and DP time: `dp_valu.counters`).
  r03_pmc_scorer_sq.json  issue / wait / LDS breakdown of k_score_ws at c4,
                  product build and chains-only diagnostic build.

SQ_INSTS_* count wave instructions; a lane-op figure is x64 (full exec mask:
an upper bound for partially active waves).  v_max_f64 is counted in the
ADD_F64 class (the DP's 3 adds + 2 maxima per cell give ~5/64 wave
instructions per cell; measured 5.5/64 at c4).

usage: scripts/pmc_fp64_summary.py [gpurun_out/r05pmc]
"""
import collections
import csv
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
FP64_LANE_OPS_PEAK = 78.6e12 / 2      # FP64 vector: 78.6 TF counts an FMA as 2 ops
F64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]


def short(name):
    return name.split("(")[0].replace("void ", "")


def dispatches(path):
    """{dispatch id: (kernel, duration ns, {counter: value})}"""
    out = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        k, _, c = out.setdefault(d, [short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), {}])
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


def fp64_pass(d, name):
    disp = dispatches(os.path.join(d, name, "p_counter_collection.csv"))
    per = collections.defaultdict(list)
    for k, dur, c in disp.values():
        per[k].append((dur, c))
    kernels = {}
    for k, lst in per.items():
        f64 = sum(sum(c.get(x, 0.0) for x in F64) for _, c in lst)
        if f64 == 0:
            continue
        dur = sum(t for t, _ in lst)
        big_t, big_c = max(lst, key=lambda x: x[0])
        big_f = sum(big_c.get(x, 0.0) for x in F64)
        kernels[k] = {
            "launches": len(lst),
            "f64_wave_insts": f64,
            "valu_wave_insts": sum(c.get("SQ_INSTS_VALU", 0.0) for _, c in lst),
            "f64_share_of_valu": f64 / max(1.0, sum(c.get("SQ_INSTS_VALU", 0.0) for _, c in lst)),
            "by_class": {x: sum(c.get(x, 0.0) for _, c in lst) for x in F64},
            "kernel_ns": dur,
            # the longest launch on its own (under PMC the launches serialise)
            "longest_launch": {"ns": big_t, "f64_wave_insts": big_f,
                               "fp64_lane_ops_per_s": big_f * 64 / (big_t * 1e-9),
                               "frac_of_fp64_peak": big_f * 64 / (big_t * 1e-9) / FP64_LANE_OPS_PEAK},
        }
    return kernels


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "r05pmc")
    out = {"source": f"scripts/pmc_fp64.sh passes c4_F / c5_F / c3_F in {os.path.relpath(d, REPO)} "
                     "(rocprofv3 --kernel-trace --pmc, one pass each); scripts/pmc_fp64_summary.py",
           "fp64_lane_ops_peak_per_s": FP64_LANE_OPS_PEAK,
           "note": "SQ_INSTS_* are wave instructions; lane-ops = x64 (full exec mask). v_max_f64 counts as ADD_F64."}
    for cfg, name in (("c4", "c4_F"), ("c5", "c5_F"), ("c3", "c3_F")):
        if not os.path.exists(os.path.join(d, name, "p_counter_collection.csv")):
            continue
        ks = fp64_pass(d, name)
        b = bench_line(os.path.join(d, name + ".log"))
        ent = {"kernels": ks}
        if cfg == "c4" and b is not None:
            # every k_dpr launch of the c4 run is the timed step's (steps 1, warmup 0, no setup realign)
            cells = b["value"] * 1e9 * b["ms_per_step"] * 1e-3
            f64 = sum(v["f64_wave_insts"] for k, v in ks.items() if k.startswith("k_dpr"))
            ent["dp"] = {"cells_per_step": cells, "f64_wave_insts_per_step": f64,
                         "f64_lane_ops_per_cell": f64 * 64 / cells,
                         "clusters": b["config"].get("clusters_per_rank", b["config"].get("clusters"))}
        out[cfg] = ent
    p = os.path.join(REPO, "profiles", "pmc_fp64.json")
    json.dump(out, open(p, "w"), indent=1)
    print("wrote", p)
    for cfg in [c for c in ("c4", "c5", "c3") if c in out]:
        for k, v in out[cfg]["kernels"].items():
            print(cfg, k, v["launches"], "%.3g" % v["f64_wave_insts"], "share %.3f" % v["f64_share_of_valu"],
                  "longest frac %.3f" % v["longest_launch"]["frac_of_fp64_peak"])
    if "dp" in out["c4"]:
        print("c4 dp", out["c4"]["dp"])

    # scorer issue breakdown (A and B counter sets, product vs chains-only)
    sq = {}
    for tag in ("ws", "chains"):
        agg = collections.defaultdict(float)
        n = 0
        for half in ("A", "B"):
            f = os.path.join(d, f"{tag}_{half}", "p_counter_collection.csv")
            if not os.path.exists(f):
                continue
            for k, dur, c in dispatches(f).values():
                if k.startswith("k_score_ws"):
                    for x, v in c.items():
                        agg[x] += v
                    if half == "A":
                        agg["kernel_ns"] += dur
                        n += 1
        if n:
            a = dict(agg)
            a["launches"] = n
            cyc = a.get("SQ_BUSY_CYCLES", 0.0) or 1.0
            wc = a.get("SQ_WAVE_CYCLES", 0.0) or 1.0
            a["derived"] = {
                "wait_inst_any_per_wave_cycle": a.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                "wait_any_per_wave_cycle": a.get("SQ_WAIT_ANY", 0.0) / wc,
                "active_inst_any_per_wave_cycle": a.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
                "lds_bank_conflict_per_lds_inst": a.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, a.get("SQ_INSTS_LDS", 1.0)),
                "f64_share_of_valu": a.get("SQ_INSTS_VALU_ADD_F64", 0.0) / max(1.0, a.get("SQ_INSTS_VALU", 1.0)),
            }
            sq[tag] = a
    if sq:
        sq["source"] = "scripts/pmc_r03.sh passes ws_A/ws_B (product) and chains_A/chains_B (librifraf_diag.so, " \
                       "RIFRAF_LEAN_NOCOMP=4: loaders skip their global loads), c4 400 clusters"
        p = os.path.join(REPO, "profiles", "r03_pmc_scorer_sq.json")
        json.dump(sq, open(p, "w"), indent=1)
        print("wrote", p)
        for tag in ("ws", "chains"):
            if tag in sq:
                print(tag, {k: round(v, 3) for k, v in sq[tag]["derived"].items()}, "ns", sq[tag]["kernel_ns"])


if __name__ == "__main__":
    main()
