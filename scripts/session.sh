#!/bin/bash
# GPU-box session steps (one parameterised script for every round-5 call;
# round 4's r04_*.sh one-offs are folded into it).  Each step runs under its
# own time limit; the first failing step ends the call.
#
# usage: scripts/session.sh TAG STEP [STEP ...]
#   tests[:K]      pytest -m gpu (optional -k filter K, ',' -> ' or ')
#   smoke          __graft_entry__.smoke()
#   bench[:ARGS]   python bench.py ARGS (',' -> ' '), line in TAG/bench.json
#   stats:CFG      rocprofv3 --kernel-trace --stats of the CFG command (c3|c4|c5)
#   pmc:CFG:CTR    one rocprofv3 --pmc pass (counters ',' separated) of CFG
#   py:SCRIPT[:ARGS] python3 SCRIPT ARGS (',' -> ' '), stdout in TAG/<name>.out
# outputs under gpurun_out/TAG/
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $D
C4="python3 bench.py --no-cpu --no-secondary --no-c3 --e2e-clusters 0 --steps 5 --warmup 2"
C5="python3 bench.py --config c5 --no-cpu --steps 5 --warmup 2"
C3="python3 scripts/c3_run.py"
cfgcmd() { case $1 in c3) echo "$C3";; c4) echo "$C4";; c5) echo "$C5";; *) echo "bad cfg $1" >&2; exit 2;; esac; }
fail() { echo "$1 failed"; tail -${3:-30} $2; exit 1; }
for step in "$@"; do
  IFS=: read -r kind a1 a2 <<< "$step"
  case $kind in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "${a1//,/ or }")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" \
        > $D/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $D/gpu_tests.log | head -20; fail tests $D/gpu_tests.log 40; }
      tail -2 $D/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 || fail smoke $D/smoke.txt
      cat $D/smoke.txt ;;
    bench)
      timeout -k 10 900 python bench.py ${a1//,/ } > $D/bench.json 2> $D/bench.err || fail bench $D/bench.err
      python3 scripts/bench_summary.py $D/bench.json ;;
    stats)
      cmd=$(cfgcmd $a1) || exit 2
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/stats_$a1 -o p --output-format csv -- $cmd \
        > $D/stats_$a1.log 2>&1 || fail "stats $a1" $D/stats_$a1.log
      echo "stats $a1 done" ;;
    pmc)
      cmd=$(cfgcmd $a1) || exit 2
      n=${a2//,/_}
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc ${a2//,/ } -d $D/pmc_$a1/$n -o p --output-format csv -- $cmd \
        > $D/pmc_${a1}_$n.log 2>&1 || fail "pmc $a1 $a2" $D/pmc_${a1}_$n.log
      echo "pmc $a1 $a2 done" ;;
    py)
      n=$(basename $a1 .py)
      timeout -k 10 900 python3 -u $a1 ${a2//,/ } > $D/$n.out 2> $D/$n.err || fail "py $a1" $D/$n.err
      tail -15 $D/$n.out ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
