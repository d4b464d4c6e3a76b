#!/bin/bash
# k_score_seg register-cap experiment: per S:WPE pair, the seg parity tests, then the c5 bench.
# usage: scripts/exp_segwpe.sh TAG S:WPE...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
for SW in "$@"; do
  export RIFRAF_SEG_S=${SW%:*} RIFRAF_SEG_WPE=${SW#*:}
  N=${SW/:/_}
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "score_dense_kernels or wide_bands" > $D/tests_$N.log 2>&1 || { echo "tests $SW failed"; tail -30 $D/tests_$N.log; exit 1; }
  tail -1 $D/tests_$N.log
  timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 3 --warmup 1 > $D/bench_$N.json 2> $D/bench_$N.err \
    || { echo "bench $SW failed"; tail -20 $D/bench_$N.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench_$N.json')); print('$SW', 'step', round(d['ms_per_step'],2), 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2))"
done
