#!/bin/bash
# c5 scorer A/B on one box: bench --config c5 with each RIFRAF_* setting given
# (alternating, two rounds).  usage: scripts/r04_ab_c5.sh TAG "ENV_A" "ENV_B" ...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
for round in 1 2; do
  i=0
  for envs in "$@"; do
    i=$((i+1))
    env $envs timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 5 --warmup 2 > $D/c5_${i}_$round.json 2> $D/c5_${i}_$round.err \
      || { echo "bench c5 [$envs] failed"; tail -20 $D/c5_${i}_$round.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$D/c5_${i}_$round.json')); print('[$envs] round $round', 'score_ms %.2f dp_ms %.2f frac %.3f parity %s' % (d['score_ms'], d['dp_ms'], d['roofline']['frac'], d['parity']['bitexact']))"
  done
done
