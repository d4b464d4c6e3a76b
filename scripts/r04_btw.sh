#!/bin/bash
# k_bt_win move buffering (BTW_MVBUF): walk/proposal parity tests, then the
# e2e native-phase timing (RIFRAF_BATCH_TIMING) with the product library and
# the per-move-store variant (librifraf_mv0.so), two rounds.  usage: TAG
set -o pipefail
TAG=${1:-r04z}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_model_e2e.py tests/test_batch.py tests/test_workloads.py \
  -m gpu -x -q --timeout 240 --timeout-method thread -k "backtrace or alignment or bt or e2e or batch or c2 or c3 or c4" \
  > $D/par.log 2>&1 || { echo "parity failed"; grep -E "FAILED|Error" $D/par.log | head; tail -30 $D/par.log; exit 1; }
tail -1 $D/par.log
for rep in 1 2; do
  for lib in hip mv0; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so RIFRAF_BATCH_TIMING=1 E2E_REPS=2 timeout -k 10 300 \
      python scripts/prof_e2e_native.py 512 > $D/e2e_${lib}_$rep.txt 2> $D/e2e_${lib}_$rep.err \
      || { echo "e2e $lib failed"; tail -20 $D/e2e_${lib}_$rep.err; exit 1; }
    echo "$lib $rep: $(grep rf_rifraf_batch $D/e2e_${lib}_$rep.err | tail -1 | cut -c1-400)"
    grep -E "^rep 1" $D/e2e_${lib}_$rep.txt
  done
done
