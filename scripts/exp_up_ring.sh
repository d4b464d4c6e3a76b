#!/bin/bash
# Pinned upload ring A/B (round 6, profiles/r08j_up_ring_ab.txt): parity of the
# product library, then configs[2] native runs with the ring (librifraf_hip)
# and with pageable copies (librifraf_noring: scripts/build_variant.sh noring
# -DRF_UP_RING=0), two alternations.
set -o pipefail
mkdir -p gpurun_out/r08j
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_batch.py tests/test_model_e2e.py > gpurun_out/r08j/par.log 2>&1 || { tail -20 gpurun_out/r08j/par.log; exit 1; }
tail -1 gpurun_out/r08j/par.log
for rep in 1 2; do
  for lib in hip noring; do
    echo -n "$lib $rep "
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 200 python scripts/c3_repeat.py 9 || exit 1
  done
done
