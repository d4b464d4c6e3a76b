#!/bin/bash
# PMC passes for the two hot kernels (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/hip
# tracing), per MI355X_MICROARCH.md §HBM / rocprofv3.  Output: gpurun_out/pmc/<tag>_*
set -e
TAG=${1:-r01}
CLU=${2:-250}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/${TAG}_${name} -o p \
    --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --clusters $CLU \
    > gpurun_out/pmc/${TAG}_${name}.log 2>&1
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run wait SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
echo "pmc done"
