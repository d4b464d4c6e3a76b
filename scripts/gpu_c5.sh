#!/bin/bash
# c5 session: bench (with CPU baseline), rocprofv3 kernel stats, PMC passes.
# usage: scripts/gpu_c5.sh TAG [extra pmc passes: inst wait lds]
set -o pipefail
TAG=${1:-r01c5}
shift || true
export TMPDIR=/tmp
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 > $D/bench.json 2> $D/bench.err \
  || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o k --output-format csv -- \
  python3 bench.py --config c5 --no-cpu --steps 2 --warmup 1 > $D/prof.log 2>&1 \
  || { echo "rocprof failed"; tail -30 $D/prof.log; exit 1; }
echo "stats done"
for p in FETCH_SIZE WRITE_SIZE "$@"; do
  case $p in
    inst) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" ;;
    wait) C="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" ;;
    lds)  C="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM TA_BUSY_avr TA_BUSY_max" ;;
    *) C=$p ;;
  esac
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $D/pmc_$p -o p --output-format csv -- \
    python3 bench.py --config c5 --no-cpu --steps 1 --warmup 1 > $D/pmc_$p.log 2>&1 \
    || { echo "pmc $p failed"; tail -20 $D/pmc_$p.log; exit 1; }
  echo "pmc $p done"
done
