#!/bin/bash
# k_bt_win window shape with the ranked walk: the product (8 elements x 16 KB),
# 6 elements per row (librifraf_wd6.so) and 16 (librifraf_wd16.so, the round-4
# walk before BTW_WD_ELEMS 8) beside the product (8); walk parity for wd6, then the e2e
# native-phase timing, two rounds.  usage: scripts/r04_btwin2.sh TAG
set -o pipefail
TAG=${1:-r04af}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_wd6.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_model_e2e.py tests/test_batch.py tests/test_frame_helpers.py -m gpu -x -q -k "backtrace or alignment or e2e or batch or frame or shift or indel" \
  --timeout 240 --timeout-method thread > $D/par_wd6.log 2>&1 \
  || { echo "wd6 parity failed"; grep -E "FAILED|Error" $D/par_wd6.log | head; tail -30 $D/par_wd6.log; exit 1; }
tail -1 $D/par_wd6.log
for rep in 1 2; do
  for v in base wd6 wd16; do
    lib=hip; env=""
    [ $v = wd6 ] && lib=wd6; [ $v = wd16 ] && lib=wd16
    [ $v = kb32 ] && env="RIFRAF_BT_WIN_KB=32"
    env $env RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so RIFRAF_BATCH_TIMING=1 E2E_REPS=2 timeout -k 10 300 \
      python scripts/prof_e2e_native.py 512 > $D/e2e_${v}_$rep.txt 2> $D/e2e_${v}_$rep.err \
      || { echo "e2e $v failed"; tail -20 $D/e2e_${v}_$rep.err; exit 1; }
    echo "$v $rep: $(grep rf_rifraf_batch $D/e2e_${v}_$rep.err | tail -1 | cut -c1-420)"
    grep -E "^rep 1" $D/e2e_${v}_$rep.txt
  done
done
