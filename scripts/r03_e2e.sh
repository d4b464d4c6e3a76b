#!/bin/bash
# e2e check: batched-driver parity tests, then the native e2e profile (1024 c4 clusters)
set -o pipefail
D=gpurun_out/${1:-r03e2e}
mkdir -p $D
[ "$2" = "notest" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_batch.py tests/test_ties.py \
  "tests/test_workloads.py::test_c4_throughput_runs_match_oracle" tests/test_gpu_parity.py::test_release_bands_then_refill tests/test_gpu_parity.py::test_validation_skip_follows_state > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
RIFRAF_BATCH_TIMING=1 E2E_REPS=3 timeout -k 10 300 python scripts/prof_e2e_native.py 1024 > $D/prof_1024.txt 2>&1 || { echo "e2e prof failed"; tail -20 $D/prof_1024.txt; exit 1; }
head -40 $D/prof_1024.txt
