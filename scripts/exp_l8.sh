#!/bin/bash
# 8-lane NP=2 DP tasks for H <= 31 (librifraf_l8b4 / l8b8: RF_OPT_DP_WIDE default 7,
# 4 or 8 periods per block): DP parity, then c4 + c5 A/B against the product.
set -o pipefail
for v in l8b4 l8b8; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads.py tests/test_golden_fixtures.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${v}_tests.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/${v}_tests.log; exit 1; }
  tail -1 gpurun_out/${v}_tests.log
done
scripts/exp_ab.sh l8ab hip l8b4 l8b8
