#!/bin/bash
# round-4 GPU session 9: the batch pipeline settings, three alternating rounds
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r04l
mkdir -p $D
S="16,1 16,2,0,256,1 16,2,0,256,0 16,3,0,128,1 16,2,0,128,1 2,1 2,2,0,256,1 2,2,0,256,0"
timeout -k 10 600 python3 scripts/e2e_pinned.py 512 $S $S $S > $D/e2e_pinned.jsonl 2> $D/e2e_pinned.err \
  || { echo "e2e pinned failed"; tail -5 $D/e2e_pinned.err; exit 1; }
python3 -c "
import json
for l in open('$D/e2e_pinned.jsonl'):
    d=json.loads(l); print(d['cores'], d['engines'], d['wave'], d['init_exclusive'], d['clusters_per_s'], d['same_consensus'], {k: d['stats'][k] for k in ('native_s','score_phase_s','setup_native_s','upload_s')})
"
