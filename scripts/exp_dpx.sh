#!/bin/bash
# scripts/exp_dpx.py under the product library and the diagnostic variants
# named on the command line (rifraf.jl_amd/librifraf_<name>.so), two rounds
# usage: scripts/exp_dpx.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
D=gpurun_out/$TAG
mkdir -p $D
for r in 1 2; do
  for v in hip "$@"; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 200 python3 scripts/exp_dpx.py >> $D/exp_dpx.jsonl 2>> $D/exp_dpx.err \
      || { echo "exp $v failed"; tail -20 $D/exp_dpx.err; exit 1; }
  done
done
cat $D/exp_dpx.jsonl
