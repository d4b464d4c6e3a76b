#!/bin/bash
# k_score_sdma vs k_score_seg at c5: parity of the wide-band scorer tests,
# then one c5 bench per variant (RIFRAF_SEG_VER / RIFRAF_SDMA_S defaults).
set -o pipefail
D=gpurun_out/${1:-r02sdma}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "wide_bands or dense_kernels or plan_cache" > $D/tests.txt 2>&1 || { echo "tests failed"; tail -30 $D/tests.txt; exit 1; }
tail -2 $D/tests.txt
for v in "2 8" "2 12" "2 16" "1 8"; do
  set -- $v
  RIFRAF_SEG_VER=$1 RIFRAF_SDMA_S=$2 timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 \
    > $D/c5_v$1_s$2.json 2> $D/c5_v$1_s$2.err || { echo "bench $v failed"; tail -20 $D/c5_v$1_s$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$D/c5_v$1_s$2.json')); print('$v', 'score_ms', round(d['score_ms'],2), 'dp_ms', round(d['dp_ms'],2), 'parity', d['parity']['bitexact'], 'gcups', round(d['value'],1))"
done
