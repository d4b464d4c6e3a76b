#!/bin/bash
# A/B of library builds on the c4 step and the c5 secondary line (no CPU
# baseline, no e2e): exp_ab.sh DIR lib1 lib2 ... (rifraf.jl_amd/librifraf_<lib>.so),
# alternated twice.  Prints dp / score ms and GCUPS per run.
set -o pipefail
D=gpurun_out/${1:-ab}; shift
mkdir -p $D
for rep in 1 2; do
  for v in "$@"; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 300 python bench.py --no-cpu --e2e-clusters 0 --steps 5 --warmup 2 \
      > $D/${v}_$rep.json 2> $D/${v}_$rep.err || { echo "bench $v failed"; tail -20 $D/${v}_$rep.err; exit 1; }
    python -c "
import json; d=json.load(open('$D/${v}_$rep.json')); s=d['secondary']
print('$v', $rep, 'c4 dp %.2f score %.2f gcups %.1f %s | c5 dp %.2f score %.2f gcups %.1f %s' % (d['dp_ms'], d['score_ms'], d['value'], d['parity']['bitexact'], s['dp_ms'], s['score_ms'], s['value'], s['parity']['bitexact']))"
  done
done
