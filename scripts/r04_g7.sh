#!/bin/bash
# round-4 GPU session 7: full GPU suite + smoke + bench; c3 A/B (64-lane
# non-lean tasks, very-wide-band DP block size); c5 A/B of the final defaults
set -o pipefail
export TMPDIR=/tmp
bash scripts/r04_check.sh r04h || exit 1
D=gpurun_out/r04h_c3ab
mkdir -p $D
for r in 1 2; do
  for s in "prod:" "nl64off:RIFRAF_DP_NL64=0" "nt256:RIFRAF_HIP_LIB=rifraf.jl_amd/librifraf_nt256.so"; do
    name=${s%%:*}; envs=${s#*:}
    timeout -k 10 300 env $envs python3 scripts/c3_run.py > $D/${name}_$r.json 2> $D/${name}_$r.err \
      || { echo "c3 $name failed"; tail -5 $D/${name}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['native_seconds_per_run'],4), d['kernel_ms_total'], d['same_as_python_stage_machine'], d['consensus_equals_template'])" $D/${name}_$r.json $name $r
  done
done
bash scripts/r04_ab_c5.sh r04h_ab "RIFRAF_SEG_COLS=64" || exit 1
