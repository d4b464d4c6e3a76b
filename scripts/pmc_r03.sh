#!/bin/bash
# Round-3 PMC passes (one rocprofv3 run per pass, --kernel-trace only):
#  A/B: issue / wait / LDS breakdown of the c4 scorer, normal and chains-only
#       (diagnostic build, RIFRAF_LEAN_NOCOMP=4);
#  F:   FP64 VALU instruction counts of every kernel at c4 and c5 (north_star:
#       the DP fill's FP64-VALU fraction from counters).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r03pmc}
mkdir -p $D
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
F="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {   # name, counters, env..., -- args
  local name=$1 ctr=$2; shift 2
  env "$@" timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $D/$name -o p --output-format csv -- \
    python3 bench.py --no-cpu --e2e-clusters 0 $BARGS > $D/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $D/$name.log; exit 1; }
  echo "pass $name done"
}
BARGS="--no-secondary --clusters 400 --steps 1 --warmup 0"
run ws_A "$A" RIFRAF_X=0
run ws_B "$B" RIFRAF_X=0
run chains_A "$A" RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_diag.so RIFRAF_LEAN_NOCOMP=4
run chains_B "$B" RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_diag.so RIFRAF_LEAN_NOCOMP=4
BARGS="--no-secondary --steps 1 --warmup 0"
run c4_F "$F" RIFRAF_X=0
BARGS="--config c5 --steps 1 --warmup 0"
run c5_F "$F" RIFRAF_X=0
