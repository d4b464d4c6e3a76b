#!/bin/bash
# One fresh-box check: GPU tests, smoke, the driver's default bench line.
# usage: scripts/round_check.sh TAG      (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-r02}
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $D/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || { echo "smoke failed"; cat $D/smoke.txt; exit 1; }
cat $D/smoke.txt
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
