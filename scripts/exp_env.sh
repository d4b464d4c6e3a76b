#!/bin/bash
# A/B timing of scorer/DP environment knobs: scripts/exp_env.sh "NAME:VAR=VAL,VAR=VAL" ...
# Output: gpurun_out/exp/NAME.json
mkdir -p gpurun_out/exp
for spec in "$@"; do
  name=${spec%%:*}
  vars=${spec#*:}
  ( IFS=','; for kv in $vars; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/exp/$name.json 2> gpurun_out/exp/$name.err ) || { echo "$name failed"; tail -5 gpurun_out/exp/$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/$name.json'));print('$name', 'dp %.2f score %.2f frac %.3f' % (d['dp_ms'], d['score_ms'], d['roofline_other']['k_score']['frac']))"
done
