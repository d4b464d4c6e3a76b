#!/bin/bash
# c5 scorer profiles for each RIFRAF_SEG_COLS value: kernel stats, FETCH_SIZE,
# SQ wait/issue counters (separate rocprofv3 runs, --kernel-trace only).
# usage: scripts/r04_prof_c5ab.sh TAG COLS...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
C5="python3 bench.py --config c5 --no-cpu --steps 3 --warmup 1"
for cols in "$@"; do
  export RIFRAF_SEG_COLS=$cols
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats_$cols -o p --output-format csv -- $C5 > $D/stats_$cols.log 2>&1 \
    || { echo "stats $cols failed"; tail -5 $D/stats_$cols.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/fetch_$cols -o p --output-format csv -- $C5 > $D/fetch_$cols.log 2>&1 \
    || { echo "fetch $cols failed"; tail -5 $D/fetch_$cols.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $D/sq_$cols -o p --output-format csv -- $C5 > $D/sq_$cols.log 2>&1 \
    || { echo "sq $cols failed"; tail -5 $D/sq_$cols.log; exit 1; }
  echo "cols $cols done"
done
