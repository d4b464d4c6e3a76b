#!/bin/bash
# k_bt_win ranked box walk (BTW_RANK, librifraf_rank.so): walk / proposal /
# e2e parity tests against the oracle and the Python stage machine, then the
# e2e native-phase timing with the product library and the variant, two
# rounds.  usage: scripts/r04_btrank.sh TAG
set -o pipefail
TAG=${1:-r04ab}
D=gpurun_out/$TAG
mkdir -p $D
export TMPDIR=/tmp
RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_rank.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_model_e2e.py tests/test_batch.py tests/test_workloads.py tests/test_frame_helpers.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $D/par_rank.log 2>&1 \
  || { echo "rank parity failed"; grep -E "FAILED|Error" $D/par_rank.log | head; tail -30 $D/par_rank.log; exit 1; }
tail -1 $D/par_rank.log
for rep in 1 2; do
  for lib in hip rank; do
    RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$lib.so RIFRAF_BATCH_TIMING=1 E2E_REPS=2 timeout -k 10 300 \
      python scripts/prof_e2e_native.py 512 > $D/e2e_${lib}_$rep.txt 2> $D/e2e_${lib}_$rep.err \
      || { echo "e2e $lib failed"; tail -20 $D/e2e_${lib}_$rep.err; exit 1; }
    echo "$lib $rep: $(grep rf_rifraf_batch $D/e2e_${lib}_$rep.err | tail -1 | cut -c1-420)"
    grep -E "^rep 1" $D/e2e_${lib}_$rep.txt
  done
done
