#!/bin/bash
# Round-3 end-of-round set at HEAD: GPU tests, smoke, default bench, rocprofv3
# kernel stats (c4, c5) and the FETCH/WRITE PMC passes.  usage: scripts/r03_final.sh TAG
set -o pipefail
TAG=${1:-r03h}
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $D/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 \
  || { echo "smoke failed"; tail -20 $D/smoke.txt; exit 1; }
cat $D/smoke.txt
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
bash scripts/prof_round.sh $TAG
