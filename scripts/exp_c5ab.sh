#!/bin/bash
# A/B of c5 (bench --config c5) over library builds: exp_c5ab.sh DIR lib1 lib2 ...
# (rifraf.jl_amd/librifraf_<lib>.so; "hip" = the product library), alternated twice.
set -o pipefail
D=gpurun_out/${1:-c5ab}; shift
mkdir -p $D
for rep in 1 2; do
  for v in "$@"; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 \
      > $D/${v}_$rep.json 2> $D/${v}_$rep.err || { echo "bench $v failed"; tail -20 $D/${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$D/${v}_$rep.json')); print('$v', $rep, 'dp_ms', round(d['dp_ms'],2), 'score_ms', round(d['score_ms'],2), 'gcups', round(d['value'],1), d['parity']['bitexact'])"
  done
done
