#!/bin/bash
set -o pipefail
D=gpurun_out/r03r_units
mkdir -p $D
RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads.py tests/test_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/par_new.log 2>&1 || { echo "parity failed"; tail -30 $D/par_new.log; exit 1; }
echo "new parity $(tail -1 $D/par_new.log)"
for rep in 1 2; do
  for lib in hip base; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 300 python bench.py --no-cpu --no-secondary --steps 5 --warmup 2 > $D/${lib}_$rep.json 2> $D/${lib}_$rep.err || { echo "$lib bench failed"; tail -10 $D/${lib}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/${lib}_$rep.json')); print('$lib $rep', 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), 'e2e', round(d['e2e']['clusters_per_s'],1), 'cold', round(d['e2e']['cold_clusters_per_s'],1), d['parity']['bitexact'], d['e2e']['same_as_python_stage_machine'])"
  done
done
