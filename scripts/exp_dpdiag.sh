#!/bin/bash
# Lean DP limiter: normal vs interior band stores sunk (RIFRAF_DP_SINK) vs
# LDS band output skipped (libdiag_b: -DDPL_NO_LDS_OUT) vs both, c4 and c5.
set -o pipefail
D=gpurun_out/${1:-r02dpdiag}
mkdir -p $D
for cfg in c4 c5; do
  extra=""; [ $cfg = c4 ] && extra="--no-secondary"
  for lib in a b; do
    for sink in 0 1; do
      f=$D/${cfg}_${lib}${sink}
      RIFRAF_DP_SINK=$sink RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/libdiag_$lib.so \
        timeout -k 10 200 python bench.py --config $cfg --no-cpu --steps 4 --warmup 1 $extra > $f.json 2> $f.err \
        || { echo "bench $f failed"; tail -20 $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f.json')); print('$cfg lib $lib sink $sink dp_ms', round(d['dp_ms'],2))"
    done
  done
done
