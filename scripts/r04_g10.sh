#!/bin/bash
# round-4 GPU session 10: device quality pass (rf_qv_probs) -- batch / workload
# GPU tests, pinned e2e settings (3 alternating rounds), the default bench line
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r04m
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_batch.py tests/test_workloads.py -m gpu -x -v --timeout 600 \
  --timeout-method thread > $D/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $D/tests.log | head; tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
S="16,1 16,2,0,256,1 2,1 2,2,0,256,1"
timeout -k 10 600 python3 scripts/e2e_pinned.py 512 $S $S $S > $D/e2e_pinned.jsonl 2> $D/e2e_pinned.err \
  || { echo "e2e pinned failed"; tail -5 $D/e2e_pinned.err; exit 1; }
python3 -c "
import json
for l in open('$D/e2e_pinned.jsonl'):
    d=json.loads(l); print(d['cores'], d['engines'], d['wave'], d['init_exclusive'], d['clusters_per_s'], d['same_consensus'], {k: d['stats'][k] for k in ('native_s','score_phase_s','setup_native_s','upload_s')})
"
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1])
e=d['e2e']; print(round(d['value'],1), e['clusters_per_s'], e['pinned'], e['same_as_python_stage_machine'], d['c3']['native_seconds_per_run'], d['c3']['same_as_python_stage_machine'])
"
