#!/bin/bash
# Full GPU suite at HEAD (k_reduce template, k_fuse), then the fused-step A/B
# with PMC (scripts/r04_fuse2.sh).  usage: scripts/r04_fuse3.sh TAG
set -o pipefail
TAG=${1:-r04s}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $D/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $D/gpu_tests.log | head; tail -30 $D/gpu_tests.log; exit 1; }
tail -2 $D/gpu_tests.log
bash scripts/r04_fuse2.sh $TAG
