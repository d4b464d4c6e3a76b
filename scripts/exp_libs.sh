#!/bin/bash
# A/B timing of experimental builds: scripts/exp_libs.sh NAME... (librifraf_NAME.so,
# "hip" = the product library).  Output: gpurun_out/exp/NAME.json
mkdir -p gpurun_out/exp
for v in "$@"; do
  export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so
  [ "$v" = hip ] && export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_hip.so
  timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/exp/$v.json 2> gpurun_out/exp/$v.err || exit 1
  echo "$v done"
done
