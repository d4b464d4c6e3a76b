#!/bin/bash
# Kernel A/B over c4 and c5: parity per library (score / DP tests), then the
# bench's DP and scoring times, two interleaved rounds on one box.
# usage: scripts/exp_ab.sh TAG name:lib[:VAR=val,...] ...   (CFGS="c4 c5" by default)
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
CFGS=${CFGS:-c4 c5}
for spec in "$@"; do
  IFS=: read name lib vars <<< "$spec"
  [ -n "$vars" ] && continue   # diagnostic builds: timing only
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_workloads.py tests/test_batch.py -m gpu -x -q --timeout 200 --timeout-method thread ${PTK:+-k "$PTK"} \
    > $D/par_$name.log 2>&1 || { echo "$name parity failed"; tail -20 $D/par_$name.log; exit 1; }
  echo "$name parity $(tail -1 $D/par_$name.log)"
done
for rep in 1 2; do
  for cfg in $CFGS; do
    for spec in "$@"; do
      IFS=: read name lib vars <<< "$spec"
      f=$D/${cfg}_${name}_$rep
      extra="--no-secondary --e2e-clusters 0"; [ $cfg = c5 ] && extra=""
      env $(echo $vars | tr ',' ' ') RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 200 python bench.py \
        --config $cfg --no-cpu $extra --steps 5 --warmup 2 > $f.json 2> $f.err \
        || { echo "$name $cfg bench failed"; tail -10 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); print('$cfg $name $rep', 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), d['parity']['bitexact'])"
    done
  done
done
