#!/bin/bash
# e2e A/B of two libraries, alternating, two rounds each
set -o pipefail
D=gpurun_out/$1
mkdir -p $D
for r in 1 2; do
  for v in hip base; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python3 -u scripts/e2e_pinned.py 512 16,2,0,256,0 \
      | sed "s/^{/{\"lib\": \"$v\", /" >> $D/e2e.jsonl 2>> $D/e2e.err || { echo "e2e $v failed"; tail -20 $D/e2e.err; exit 1; }
  done
done
