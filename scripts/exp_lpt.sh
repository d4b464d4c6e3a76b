#!/bin/bash
# 64-lane DP tasks: parity (default RIFRAF_DP_WIDE=1 and =3) then DP-only timing
# against the product library.  Stops at the first failure.
set -o pipefail
L=$PWD/rifraf.jl_amd/librifraf_lpt.so
RIFRAF_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lpt_tests.log 2>&1 || { echo "lpt tests failed"; tail -30 gpurun_out/lpt_tests.log; exit 1; }
tail -1 gpurun_out/lpt_tests.log
RIFRAF_DP_WIDE=3 RIFRAF_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dp_" > gpurun_out/lpt3_tests.log 2>&1 || { echo "lpt3 tests failed"; tail -30 gpurun_out/lpt3_tests.log; exit 1; }
tail -1 gpurun_out/lpt3_tests.log
for rep in 1 2; do
for v in hip lpt lpt3; do
  lib=$v; env=""; [ $v = lpt3 ] && { lib=lpt; env="RIFRAF_DP_WIDE=3"; }
  env $env RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 200 python scripts/exp_dp_only.py 18 > gpurun_out/dp_$v.json 2>gpurun_out/dp_$v.err || { echo "$v failed"; tail -5 gpurun_out/dp_$v.err; exit 1; }
  echo "$v $rep $(cat gpurun_out/dp_$v.json)"
done
done
