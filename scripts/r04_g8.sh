#!/bin/bash
# round-4 GPU session 8: the batch pipeline (waves from a shared queue, at most
# one engine in its native stage machine) at 16 and 2 host cores; the GPU
# tests of the batch driver
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r04j
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_batch.py -m gpu -x -v --timeout 240 --timeout-method thread \
  > $D/batch_tests.log 2>&1 || { echo "batch tests failed"; tail -30 $D/batch_tests.log; exit 1; }
tail -2 $D/batch_tests.log
timeout -k 10 600 python3 scripts/e2e_pinned.py 512 16,1 2,1 16,2,0,128,1 2,2,0,128,1 16,2,0,64,1 2,2,0,64,1 \
  16,2,0,128,0 2,2,0,128,0 2,2,1,128,1 16,3,0,64,1 2,3,0,64,1 16,2,0,256,1 2,2,0,256,1 \
  > $D/e2e_pinned.jsonl 2> $D/e2e_pinned.err || { echo "e2e pinned failed"; tail -5 $D/e2e_pinned.err; exit 1; }
python3 -c "
import json
for l in open('$D/e2e_pinned.jsonl'):
    d=json.loads(l); print(d['cores'], d['engines'], d['sync_block'], d['wave'], d['init_exclusive'], d['clusters_per_s'], d['same_consensus'])
"
