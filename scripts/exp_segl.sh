#!/bin/bash
# k_score_segl at c5: default build, diagnostic build with the chains skipped
# (RIFRAF_LEAN_NOCOMP=1) or the segment loads skipped (=2), and variant builds
# (librifraf_<tag>.so, e.g. -DSEGL_UNROLL / -DSEGL_FENCE_KIND): exp_segl.sh DIR [tag ...]
set -o pipefail
D=gpurun_out/${1:-r02segl}; shift
mkdir -p $D
run() {   # tag lib [VAR=val ...]
  local tag=$1 lib=$2; shift 2
  env "$@" RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/$lib timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 \
    > $D/$tag.json 2> $D/$tag.err || { echo "bench $tag failed"; tail -20 $D/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$D/$tag.json')); print('$tag', 'dp_ms', round(d['dp_ms'],2), 'score_ms', round(d['score_ms'],2), d['parity']['bitexact'])"
}
run base librifraf_hip.so
run nochain librifraf_diag.so RIFRAF_LEAN_NOCOMP=1
run noload librifraf_diag.so RIFRAF_LEAN_NOCOMP=2
for t in "$@"; do run $t librifraf_$t.so; done
