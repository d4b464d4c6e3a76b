#!/bin/bash
# Same-box A/B of the c4 bench under environment settings, alternating:
# exp_ab.sh DIR ROUNDS "tagA=VAR=val,..." "tagB=VAR=val,..." ...
set -o pipefail
D=gpurun_out/${1:-r02ab}; R=${2:-2}; shift 2
mkdir -p $D
for r in $(seq 1 $R); do
  for spec in "$@"; do
    tag=${spec%%=*}; vars=${spec#*=}
    f=$D/${tag}_$r
    env $(echo $vars | tr ',' ' ') timeout -k 10 200 python bench.py --no-cpu --no-secondary --e2e-clusters 0 --steps 10 --warmup 3 > $f.json 2> $f.err \
      || { echo "bench $tag failed"; tail -20 $f.err; exit 1; }
    python -c "import json; d=json.load(open('$f.json')); print('$tag', $r, 'value', round(d['value'],1), 'dp_ms', round(d['dp_ms'],2), 'score_ms', round(d['score_ms'],2))"
  done
done
