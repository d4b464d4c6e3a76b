#!/bin/bash
# Round-4 GPU session: parity tests (-m gpu, optionally a -k filter), smoke,
# default bench.  usage: scripts/r04_check.sh TAG [tests|notests] [PYTEST_K]
set -o pipefail
TAG=${1:-r04}
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
if [ "${2:-tests}" = "tests" ]; then
  K=()
  [ -n "$3" ] && K=(-k "$3")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
    > $D/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" $D/gpu_tests.log | head -20; tail -40 $D/gpu_tests.log; exit 1; }
  tail -3 $D/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 \
    || { echo "smoke failed"; tail -20 $D/smoke.txt; exit 1; }
  cat $D/smoke.txt
fi
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
python - $D/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d.get("secondary", {})
print({k: d.get(k) for k in ("value", "ms_per_step", "dp_ms", "score_ms")}, d["roofline"]["frac"])
print("c5", {k: s.get(k) for k in ("value", "dp_ms", "score_ms")}, s.get("roofline", {}).get("frac"), s.get("roofline", {}).get("traffic"))
print("e2e", {k: d.get("e2e", {}).get(k) for k in ("clusters_per_s", "consensus_equals_template", "same_as_python_stage_machine")})
PY
