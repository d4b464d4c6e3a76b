#!/bin/bash
# round-4 end-of-round set at HEAD: GPU tests, smoke, default bench
# (r04_check.sh), then 2-rank rehearsals of the c4 and c5 bench lines on the
# one GPU (gloo, --shared-gpu).  usage: scripts/r04_final.sh TAG
set -o pipefail
TAG=${1:-r04k}
D=gpurun_out/$TAG
export TMPDIR=/tmp
bash scripts/r04_check.sh $TAG || exit 1
for cfg in c4 c5; do
  timeout -k 10 900 python bench.py --gpus 2 --shared-gpu --backend gloo --config $cfg --no-cpu --steps 3 --warmup 1 \
    > $D/${cfg}_2ranks.json 2> $D/${cfg}_2ranks.err || { echo "$cfg 2 ranks failed"; tail -20 $D/${cfg}_2ranks.err; exit 1; }
  python3 - $D/${cfg}_2ranks.json <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]).read().splitlines() if l.strip()]
d = json.loads(lines[-1])
e = d.get("e2e") or {}
s = d.get("sharded_rifraf") or {}
print(d["config"]["workload"], d["n_gpus"], round(d["value"], 1), d["scaling"], "lines", len(lines),
      "e2e", e.get("ranks"), e.get("clusters_per_s"), (e.get("pinned") or {}).get("ratio_to_unpinned"),
      "sharded", s.get("exchange_ms_per_iteration"), s.get("same_as_one_gpu"))
PY
done
