#!/bin/bash
# DP variants A/B at the c4 shape: parity (DP + c4 dense tests) per library,
# then interleaved DP-only timings.  usage: scripts/exp_dp_ab.sh TAG lib1 lib2 ...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
for v in "$@"; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_workloads.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dp_ or c4_clusters or bands" \
    > $D/par_$v.log 2>&1 || { echo "$v parity failed"; tail -20 $D/par_$v.log; exit 1; }
  echo "$v parity $(tail -1 $D/par_$v.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python scripts/exp_dp_c4.py > $D/dp_${v}_$rep.json 2> $D/dp_$v.err \
      || { echo "$v timing failed"; tail -5 $D/dp_$v.err; exit 1; }
    echo "$v $rep $(cat $D/dp_${v}_$rep.json)"
  done
done
