#!/bin/bash
# e2e + c4 under engine environment options: exp_e2e_env.sh TAG name=VAR=val,... ...
set -o pipefail
D=gpurun_out/$1; shift
mkdir -p $D
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; vars=${spec#*=}
    env $(echo $vars | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 5 --warmup 2 > $D/${name}_$rep.json 2> $D/${name}_$rep.err || { echo "$name failed"; tail -10 $D/${name}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/${name}_$rep.json')); print('$name $rep', 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'e2e', round(d['e2e']['clusters_per_s'],1), 'cold', round(d['e2e']['cold_clusters_per_s'],1), d['parity']['bitexact'], d['e2e']['same_as_python_stage_machine'])"
  done
done
