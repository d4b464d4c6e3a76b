#!/bin/bash
# Round-4 closing check with the ranked walk: GPU suite, smoke, bench line
# (scripts/r04_check.sh), then the c3 field with the sequential walk
# (librifraf_seqwalk.so) beside the product's.  usage: scripts/r04_close.sh TAG
set -o pipefail
TAG=${1:-r04ac}
D=gpurun_out/$TAG
bash scripts/r04_check.sh $TAG || exit 1
for lib in hip seqwalk; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so timeout -k 10 300 python bench.py --no-cpu --no-secondary \
    --e2e-clusters 0 --steps 3 --warmup 1 > $D/c3_$lib.json 2> $D/c3_$lib.err || { echo "c3 $lib failed"; tail -20 $D/c3_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/c3_$lib.json'))['c3']; print('$lib c3', {k: d.get(k) for k in ('seconds', 'runs_per_s', 'bt_ms', 'backtrace_ms', 'kernel_ms')})"
done
