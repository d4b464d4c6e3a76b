#!/bin/bash
# 32-lane DP tasks for H 64..127 (librifraf_l32.so: RF_OPT_DP_WIDE default 3):
# parity, then DP-only and c5 timing against the product library.
set -o pipefail
L=$PWD/rifraf.jl_amd/librifraf_l32.so
RIFRAF_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/l32_tests.log 2>&1 || { echo "l32 tests failed"; tail -30 gpurun_out/l32_tests.log; exit 1; }
tail -1 gpurun_out/l32_tests.log
for rep in 1 2; do
for v in hip l32; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python scripts/exp_dp_only.py 18 > gpurun_out/dp_$v.json 2>gpurun_out/dp_$v.err || { echo "$v failed"; tail -5 gpurun_out/dp_$v.err; exit 1; }
  echo "$v $rep $(cat gpurun_out/dp_$v.json)"
done
done
