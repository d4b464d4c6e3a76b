#!/bin/bash
# e2e field of the c4 bench at several engine counts: exp_e2e.sh DIR CLUSTERS E1 E2 ...
set -o pipefail
D=gpurun_out/${1:-e2e}; N=$2; shift 2
mkdir -p $D
for e in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 1 --warmup 1 --clusters 64 --e2e-clusters $N --e2e-engines $e \
    > $D/e$e.json 2> $D/e$e.err || { echo "e2e $e failed"; tail -20 $D/e$e.err; exit 1; }
  python -c "import json; d=json.load(open('$D/e$e.json'))['e2e']; print('engines', $e, 'clusters/s', round(d['clusters_per_s'],1), d['same_as_python_stage_machine'], d['consensus_equals_template'])"
done
