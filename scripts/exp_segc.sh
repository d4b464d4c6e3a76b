#!/bin/bash
# wide-band scorer variants at c5 (RIFRAF_SEG_VER / RIFRAF_SEG_S defaults), after their parity tests;
# with DIAG=1 also segc's loads-only / chains-only times (librifraf_diag.so)
set -o pipefail
D=gpurun_out/${1:-r02segc}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "wide_bands or dense_kernels or plan_cache" > $D/tests.txt 2>&1 || { echo "tests failed"; tail -30 $D/tests.txt; exit 1; }
tail -1 $D/tests.txt
for v in ${VARIANTS:-"3 16" "3 24" "3 32" "1 24"}; do :; done
for v in "3 16" "3 24" "3 32" "1 24"; do
  set -- $v
  RIFRAF_SEG_VER=$1 RIFRAF_SEG_S=$2 timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 \
    > $D/c5_v$1_s$2.json 2> $D/c5_v$1_s$2.err || { echo "bench $v failed"; tail -20 $D/c5_v$1_s$2.err; exit 1; }
  python -c "import json; d=json.load(open('$D/c5_v$1_s$2.json')); print('$v', 'score_ms', round(d['score_ms'],2), 'parity', d['parity']['bitexact'])"
done
if [ -n "$DIAG" ]; then
  for f in 1 2; do
    RIFRAF_SEG_VER=3 RIFRAF_SEG_S=${DIAG} RIFRAF_LEAN_NOCOMP=$f RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_diag.so \
      timeout -k 10 200 python bench.py --config c5 --no-cpu --steps 4 --warmup 1 > $D/c5_diag$f.json 2> $D/c5_diag$f.err \
      || { echo "diag $f failed"; exit 1; }
    python -c "import json; d=json.load(open('$D/c5_diag$f.json')); print('diag $f score_ms', round(d['score_ms'],2))"
  done
fi
