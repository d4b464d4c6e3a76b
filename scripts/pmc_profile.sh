#!/bin/bash
# PMC passes for the hot kernels (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/hip
# tracing), per MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots (FETCH_SIZE and
# WRITE_SIZE cannot share a pass).  Output: gpurun_out/pmc/<tag>_<pass>/
# usage: scripts/pmc_profile.sh TAG CLUSTERS [passes...]   (default: fetch write)
set -e
TAG=${1:-r01}
CLU=${2:-250}
shift 2 || true
PASSES=${@:-fetch write}
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for p in $PASSES; do
  case $p in
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE" ;;
    inst)  C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" ;;
    wait)  C="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" ;;
    lds)   C="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM TA_BUSY_avr TA_BUSY_max" ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc/${TAG}_$p -o p \
    --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --clusters $CLU \
    > gpurun_out/pmc/${TAG}_$p.log 2>&1
  echo "pass $p done"
done
