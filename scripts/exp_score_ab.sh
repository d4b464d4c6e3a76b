#!/bin/bash
# Scorer A/B at c4: parity per library (score tests), then bench scoring
# times.  usage: scripts/exp_score_ab.sh TAG name:lib[:VAR=val,...] ...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
for spec in "$@"; do
  IFS=: read name lib vars <<< "$spec"
  [ -n "$vars" ] && continue   # diagnostic builds: timing only
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_workloads.py tests/test_batch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "score or c4 or native" \
    > $D/par_$name.log 2>&1 || { echo "$name parity failed"; tail -20 $D/par_$name.log; exit 1; }
  echo "$name parity $(tail -1 $D/par_$name.log)"
done
for rep in 1 2; do
  for spec in "$@"; do
    IFS=: read name lib vars <<< "$spec"
    f=$D/${name}_$rep
    env $(echo $vars | tr ',' ' ') RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 200 python bench.py \
      --no-cpu --no-secondary --e2e-clusters 0 --steps 5 --warmup 2 > $f.json 2> $f.err \
      || { echo "$name bench failed"; tail -10 $f.err; exit 1; }
    python -c "import json; d=json.load(open('$f.json')); print('$name $rep', 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), d['parity']['bitexact'])"
  done
done
