#!/bin/bash
# One GPU session: parity tests, bench (with CPU baseline), rocprofv3 kernel stats,
# PMC FETCH/WRITE passes.  usage: scripts/gpu_check.sh TAG [CLUSTERS]
set -o pipefail
TAG=${1:-r01}
CLU=${2:-1250}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$TAG/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o k --output-format csv -- \
  python3 bench.py --no-cpu --steps 5 --warmup 2 --clusters $CLU > gpurun_out/$TAG/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/$TAG/prof.log; exit 1; }
echo "stats done"
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $p -d gpurun_out/$TAG/pmc_$p -o p --output-format csv -- \
    python3 bench.py --no-cpu --steps 1 --warmup 1 --clusters $CLU > gpurun_out/$TAG/pmc_$p.log 2>&1 || { echo "pmc $p failed"; tail -20 gpurun_out/$TAG/pmc_$p.log; exit 1; }
  echo "pmc $p done"
done
