#!/bin/bash
# k_score_seg occupancy experiment: c5 bench per RIFRAF_SEG_LDS pad (bytes).
# usage: scripts/exp_seglds.sh TAG PAD...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
for L in "$@"; do
  export RIFRAF_SEG_LDS=$L
  timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 3 --warmup 1 > $D/bench_$L.json 2> $D/bench_$L.err \
    || { echo "bench $L failed"; tail -20 $D/bench_$L.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$L.json')); print('pad=$L', 'step', round(d['ms_per_step'],2), 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2))"
done
