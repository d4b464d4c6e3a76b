#!/bin/bash
# Round-3 GPU session: parity tests, smoke, default bench, self-launched
# 2-rank rehearsal (two ranks on the box's one GPU), FP64 counter names.
# usage: scripts/r03_check.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r03}
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $D/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $D/gpu_tests.log; exit 1; }
  tail -2 $D/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 \
    || { echo "smoke failed"; tail -20 $D/smoke.txt; exit 1; }
  cat $D/smoke.txt
fi
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 python bench.py --gpus 2 --shared-gpu --backend gloo --clusters 200 --e2e-clusters 32 --no-cpu \
  > $D/bench_2ranks.json 2> $D/bench_2ranks.err || { echo "2-rank bench failed"; tail -30 $D/bench_2ranks.err; exit 1; }
cat $D/bench_2ranks.json
timeout -k 10 120 rocprofv3 --list-avail > $D/list_avail.txt 2>&1 || true
grep -i "f64\|fp64" $D/list_avail.txt | head -40 || true
