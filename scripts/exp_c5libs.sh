#!/bin/bash
# c5 timing of experimental builds: scripts/exp_c5libs.sh NAME... -> gpurun_out/exp/c5_NAME.json
mkdir -p gpurun_out/exp
for v in "$@"; do
  export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so
  [ "$v" = hip ] && export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_hip.so
  timeout -k 10 300 python bench.py --config c5 --no-cpu --steps 2 --warmup 1 > gpurun_out/exp/c5_$v.json 2> gpurun_out/exp/c5_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp/c5_$v.json'));print('c5 $v', 'dp %.2f score %.2f value %.1f' % (d['dp_ms'], d['score_ms'], d['value']))"
done
