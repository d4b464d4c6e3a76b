#!/bin/bash
# Round profiles on the GPU box: rocprofv3 --kernel-trace --stats of the c4 and
# c5 bench commands, then one PMC pass each for FETCH_SIZE and WRITE_SIZE
# (separate runs, --kernel-trace only; MI355X_MICROARCH.md §HBM).
# usage: scripts/prof_round.sh TAG [CONFIGS] [COUNTERS]   (outputs under gpurun_out/TAG/)
#   CONFIGS default "c4 c5", COUNTERS default "FETCH_SIZE WRITE_SIZE"
set -o pipefail
TAG=${1:-r02}
CFGS=${2:-"c4 c5"}
CTRS=${3:-"FETCH_SIZE WRITE_SIZE"}
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
C4="python3 bench.py --no-cpu --no-secondary --no-c3 --e2e-clusters 0 --steps 5 --warmup 2"
C5="python3 bench.py --config c5 --no-cpu --steps 5 --warmup 2"
run() {   # name, rocprof args..., -- command
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" > $D/$name.log 2>&1 || { echo "$name failed"; tail -5 $D/$name.log; exit 1; }
  echo "$name done"
}
for cfg in $CFGS; do
  cmd=$C4; [ $cfg = c5 ] && cmd=$C5
  run stats_$cfg --kernel-trace --stats -d $D/stats_$cfg -o p --output-format csv -- $cmd
done
for cfg in $CFGS; do
  cmd=$C4; [ $cfg = c5 ] && cmd=$C5
  for ctr in $CTRS; do
    run pmc_${cfg}_$ctr --kernel-trace --pmc $ctr -d $D/pmc_$cfg/pmc_$ctr -o p --output-format csv -- $cmd
  done
done
