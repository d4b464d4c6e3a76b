#!/bin/bash
# k_bt_win window size at c5 (band-doubling backtraces + alignment_proposals), after the backtrace tests
set -o pipefail
D=gpurun_out/${1:-r02bt}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "backtrace or alignment_proposals" > $D/tests.txt 2>&1 || { echo "tests failed"; tail -30 $D/tests.txt; exit 1; }
tail -1 $D/tests.txt
for kb in 32 16; do
  RIFRAF_BT_WIN_KB=$kb timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 2 --warmup 1 > $D/c5_bt$kb.json 2> $D/c5_bt$kb.err \
    || { echo "bench $kb failed"; tail -20 $D/c5_bt$kb.err; exit 1; }
  python -c "import json; d=json.load(open('$D/c5_bt$kb.json')); b=d['band_doubling']; print('$kb', 'bt_ms', round(b['backtrace_ms_rank0'],2), 'rounds', b['rounds_rank0'], 'aln_ms', round(d['alignment_proposals_ms_rank0'],2), 'score_ms', round(d['score_ms'],2))"
done
