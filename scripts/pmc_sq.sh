#!/bin/bash
# SQ / LDS PMC passes (one rocprofv3 run each, --kernel-trace only) for the
# c4 and c5 bench kernels: issue vs wait vs LDS-conflict breakdown.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${1:-r02sq}
mkdir -p $D
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
for cfg in ${CFGS:-c5 c4}; do
  extra=""; [ $cfg = c4 ] && extra="--no-secondary --clusters 400"
  for p in A B; do
    C=${!p}
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C -d $D/${cfg}_$p -o p --output-format csv -- \
      python3 bench.py --config $cfg --no-cpu --steps 1 --warmup 0 $extra > $D/${cfg}_$p.log 2>&1 \
      || { echo "pass $cfg $p failed"; tail -5 $D/${cfg}_$p.log; exit 1; }
    echo "pass $cfg $p done"
  done
done
