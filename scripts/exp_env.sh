#!/bin/bash
# bench.py under alternative engine options: exp_env.sh <tag>=<VAR=val,...> ...
# (c4 unless CFG is set; results under gpurun_out/$DIR)
set -o pipefail
D=gpurun_out/${DIR:-r02env}
mkdir -p $D
CFG=${CFG:-c4}
for spec in "$@"; do
  tag=${spec%%=*}; vars=${spec#*=}
  f=$D/${CFG}_$tag
  extra=""; [ $CFG = c4 ] && extra="--no-secondary"
  env $(echo $vars | tr ',' ' ') timeout -k 10 200 python bench.py --config $CFG --no-cpu --steps 5 --warmup 2 $extra > $f.json 2> $f.err \
    || { echo "bench $tag failed"; tail -20 $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f.json')); print('$tag', 'dp_ms', round(d['dp_ms'],2), 'score_ms', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), d['parity']['bitexact'])"
done
