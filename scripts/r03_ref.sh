#!/bin/bash
# native reference-guided batches: batch tests (hub / oracle parity), then c3 throughput with the native run
set -o pipefail
D=gpurun_out/${1:-r03ref}
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_batch.py \
  > $D/batch.log 2>&1 || { echo "batch tests failed"; tail -60 $D/batch.log; exit 1; }
tail -3 $D/batch.log
timeout -k 10 600 python scripts/e2e_ref.py 64 > $D/e2e_ref.json 2> $D/e2e_ref.err || { echo "e2e_ref failed"; tail -30 $D/e2e_ref.err; exit 1; }
cat $D/e2e_ref.json
[ "$2" = "c3" ] || exit 0
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
  "tests/test_workloads.py::test_c3_throughput_frame_run_matches_oracle" > $D/c3.log 2>&1 || { echo "c3 failed"; tail -60 $D/c3.log; exit 1; }
tail -3 $D/c3.log
