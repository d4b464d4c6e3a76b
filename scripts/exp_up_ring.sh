#!/bin/bash
# Host-transfer A/B on configs[2] (round 6): parity of the product library,
# then native c3 runs (scripts/c3_repeat.py, median of 9) for each library
# named, two alternations.  r08j: the pinned upload ring (librifraf_hip vs
# librifraf_noring, built with -DRF_UP_RING=0); r08k: pinned download landing
# (librifraf_hip vs librifraf_base, the previous commit).
# usage: scripts/exp_up_ring.sh TAG lib [lib ...]
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_batch.py tests/test_model_e2e.py > gpurun_out/$TAG/par.log 2>&1 || { tail -20 gpurun_out/$TAG/par.log; exit 1; }
tail -1 gpurun_out/$TAG/par.log
for rep in 1 2; do
  for lib in "$@"; do
    echo -n "$lib $rep "
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 200 python scripts/c3_repeat.py 9 || exit 1
  done
done
