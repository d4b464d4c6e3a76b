#!/bin/bash
# product parity on the restructured segl + new upload path, then the c4 scorer A/B
set -o pipefail
mkdir -p gpurun_out/scab1
[ -n "$SKIP_PAR" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_workloads.py tests/test_batch.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "wide or score or c5 or codes or aln_error or native" > gpurun_out/scab1/par_product.log 2>&1 \
  || { echo "product parity failed"; tail -30 gpurun_out/scab1/par_product.log; exit 1; }
echo "product parity $(tail -1 gpurun_out/scab1/par_product.log)"
bash scripts/exp_score_ab.sh scab1 ws:hip w2n6:w2n6 w2n7:w2n7 loads:diag:RIFRAF_LEAN_NOCOMP=1 chains:diag:RIFRAF_LEAN_NOCOMP=4
