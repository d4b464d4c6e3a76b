#!/bin/bash
# k_score_seg (register-staged) at c5: normal vs chains skipped vs loads
# skipped (diagnostic build librifraf_diag.so, RIFRAF_LEAN_NOCOMP bits).
set -o pipefail
D=gpurun_out/${1:-r02segdiag}
mkdir -p $D
for v in 0 1 2; do
  RIFRAF_SEG_VER=1 RIFRAF_LEAN_NOCOMP=$v RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_diag.so \
    timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 > $D/c5_diag$v.json 2> $D/c5_diag$v.err \
    || { echo "bench $v failed"; tail -20 $D/c5_diag$v.err; exit 1; }
  python -c "import json; d=json.load(open('$D/c5_diag$v.json')); print('diag $v score_ms', round(d['score_ms'],2))"
done
