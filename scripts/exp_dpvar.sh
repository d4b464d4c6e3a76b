#!/bin/bash
# c4 DP time of build variants rifraf.jl_amd/libdp_<v>.so (bench parity included).
set -o pipefail
D=gpurun_out/${DIR:-r02dpvar}
mkdir -p $D
CFG=${CFG:-c4}
for v in "$@"; do
  f=$D/${CFG}_$v
  extra=""; [ $CFG = c4 ] && extra="--no-secondary"
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/libdp_$v.so timeout -k 10 200 python bench.py --config $CFG --no-cpu --steps 5 --warmup 2 $extra > $f.json 2> $f.err \
    || { echo "bench $v failed"; tail -20 $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f.json')); print('$v', 'dp_ms', round(d['dp_ms'],2), 'score_ms', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), d['parity']['bitexact'])"
done
