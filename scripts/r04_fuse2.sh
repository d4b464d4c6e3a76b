#!/bin/bash
# Fused-step prototype A/B: parity of both k_fuse builds (interior fast path
# on = product, off = librifraf_nofast.so), then the c4 bench step: product
# A/B fill + scoring vs B fill + k_fuse (fast, nofast), two interleaved
# rounds on one box; rocprofv3 kernel stats of the fused step.
# usage: scripts/r04_fuse2.sh TAG
set -o pipefail
TAG=${1:-r04p}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
for lib in hip nofast; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 400 python -u -m pytest tests/test_fuse.py -x -v \
    --timeout 200 --timeout-method thread > $D/fuse_tests_$lib.log 2>&1 \
    || { echo "fuse tests ($lib) failed"; tail -40 $D/fuse_tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $D/fuse_tests_$lib.log)"
done
for rep in 1 2; do
  for v in base fwd fwdnofast; do
    extra=""; lib=hip
    [ $v = fwd ] && extra="--score-fwd"
    [ $v = fwdnofast ] && { extra="--score-fwd"; lib=nofast; }
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 300 python bench.py --no-cpu --no-secondary \
      --no-c3 --e2e-clusters 0 --steps 5 --warmup 2 $extra > $D/c4_${v}_$rep.json 2> $D/c4_${v}_$rep.err \
      || { echo "bench $v failed"; tail -20 $D/c4_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$D/c4_${v}_$rep.json')); print('$v $rep', 'value', round(d['value'],1), 'dp', round(d['dp_ms'],2), 'score', round(d['score_ms'],2), 'step', round(d['ms_per_step'],2), d['parity']['bitexact'])"
  done
done
C4F="python3 bench.py --no-cpu --no-secondary --no-c3 --e2e-clusters 0 --steps 5 --warmup 2 --score-fwd"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/stats_fwd -o p --output-format csv -- $C4F \
  > $D/stats_fwd.log 2>&1 || { echo "rocprof stats failed"; tail -20 $D/stats_fwd.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $D/pmc_fwd/pmc_$ctr -o p --output-format csv -- $C4F \
    > $D/pmc_fwd_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -20 $D/pmc_fwd_$ctr.log; exit 1; }
done
find $D -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | head
