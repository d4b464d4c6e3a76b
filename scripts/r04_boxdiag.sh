#!/bin/bash
# Box diagnostics for the c4 DP's box-to-box spread (8.3 / 9.3 ms): the bench
# line with its write-bandwidth probe, rocm-smi clocks, and one PMC pass of
# GRBM_GUI_ACTIVE (GPU busy cycles -> effective clock per kernel).
# usage: scripts/r04_boxdiag.sh TAG
set -o pipefail
TAG=${1:-r04u}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
(rocm-smi --showclocks --showpower --showmemuse 2>&1 || true) > $D/smi.txt
C4="python3 bench.py --no-cpu --no-secondary --no-c3 --e2e-clusters 0 --steps 5 --warmup 2"
timeout -k 10 300 $C4 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench.json')); print('dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'read', round(d['stream_read_gbs']), 'write', d.get('stream_write_gbs'))"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $D/pmc -o p --output-format csv -- $C4 \
  > $D/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $D/pmc.log; exit 1; }
python3 - $D <<'PY'
import csv, collections, glob, sys
D = sys.argv[1]
f = glob.glob(D + "/pmc/**/*counter_collection.csv", recursive=True)[0]
kt = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    d = int(r["Dispatch_Id"])
    kt.setdefault((k, d), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    kt[(k, d)]["ns"] = float(r.get("End_Timestamp", 0)) - float(r.get("Start_Timestamp", 0))
agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
for (k, d), v in kt.items():
    if "GRBM_GUI_ACTIVE" in v and v["ns"] > 0:
        a = agg[k]; a[0] += v["GRBM_GUI_ACTIVE"]; a[1] += v["ns"]; a[2] += 1
for k, (c, ns, n) in sorted(agg.items(), key=lambda x: -x[1][1])[:8]:
    print(k[:40], n, "ms", round(ns / n / 1e6, 3), "GHz", round(c / ns, 3))
PY
# the fused step on 1 and 2 free-running contexts (k_fuse beside the B fill)
for fwd in 0 1; do
  SCORE_FWD=$fwd ENGINES=1,2 STEPS=8 timeout -k 10 400 python3 scripts/exp_overlap.py > $D/overlap_fwd$fwd.jsonl 2> $D/overlap_fwd$fwd.err \
    || { echo "overlap $fwd failed"; tail -20 $D/overlap_fwd$fwd.err; exit 1; }
  cat $D/overlap_fwd$fwd.jsonl
done
