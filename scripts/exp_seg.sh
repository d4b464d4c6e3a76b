#!/bin/bash
# k_score_seg experiments: parity of the seg configs, then c5 bench per RIFRAF_SEG_S value
# and one FETCH_SIZE pass each.  usage: scripts/exp_seg.sh TAG S...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "score_dense_kernels or wide_bands" > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for S in "$@"; do
  export RIFRAF_SEG_S=$S
  timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 3 --warmup 1 > $D/bench_$S.json 2> $D/bench_$S.err \
    || { echo "bench $S failed"; tail -20 $D/bench_$S.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/bench_$S.json')); print('S=$S', 'step', round(d['ms_per_step'],2), 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2))"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/pmc_$S -o p --output-format csv -- \
    python3 bench.py --config c5 --no-cpu --steps 1 --warmup 0 > $D/pmc_$S.log 2>&1 || { echo "pmc $S failed"; tail -20 $D/pmc_$S.log; exit 1; }
  python3 - $D/pmc_$S/p_counter_collection.csv <<'PY'
import csv, collections, sys
d = collections.defaultdict(float); nm = {}
for r in csv.DictReader(open(sys.argv[1])):
    i = int(r["Dispatch_Id"]); d[i] += float(r["Counter_Value"]); nm[i] = r["Kernel_Name"].split("(")[0]
for i in sorted(d):
    if "score" in nm[i]:
        print("  ", nm[i], "FETCH raw GB", round(d[i] * 1024 / 1e9, 1))
PY
done
