#!/bin/bash
# FP64 VALU counter passes (north_star: the DP fill's FP64-VALU fraction from
# counters), one rocprofv3 --kernel-trace --pmc run per config: c4 and c5 (one
# timed step, no warm-up) and configs[2] (scripts/c3_run.py).  Summarised by
# scripts/pmc_fp64_summary.py gpurun_out/TAG into profiles/pmc_fp64.json.
# usage: scripts/pmc_fp64.sh TAG
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r05pmc}
mkdir -p $D
F="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {   # name, -- command
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $F -d $D/$name -o p --output-format csv -- "$@" \
    > $D/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $D/$name.log; exit 1; }
  echo "pass $name done"
}
run c4_F python3 bench.py --no-cpu --no-secondary --no-c3 --e2e-clusters 0 --steps 1 --warmup 0
run c5_F python3 bench.py --config c5 --no-cpu --steps 1 --warmup 0
run c3_F python3 scripts/c3_run.py
