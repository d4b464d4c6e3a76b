#!/bin/bash
# DP-only timing at the c5 shape over library builds: exp_dp_libs.sh BW lib1 lib2 ...
set -o pipefail
BW=$1; shift
mkdir -p gpurun_out/dp
for rep in 1 2; do
  for v in "$@"; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python scripts/exp_dp_only.py $BW \
      > gpurun_out/dp/${v}_$BW_$rep.json 2>gpurun_out/dp/${v}.err || { echo "$v failed"; tail -5 gpurun_out/dp/${v}.err; exit 1; }
    echo "$v $rep $(cat gpurun_out/dp/${v}_$BW_$rep.json)"
  done
done
