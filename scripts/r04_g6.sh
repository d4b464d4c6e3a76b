#!/bin/bash
# round-4 GPU session: full GPU suite, smoke, bench; c5 SEGL_MASKED_MIN A/B;
# c3 kernel stats; pinned-core e2e settings
set -o pipefail
export TMPDIR=/tmp
bash scripts/r04_check.sh r04g || exit 1
bash scripts/r04_ab_c5.sh r04g_ab "RIFRAF_SEG_COLS=64" "RIFRAF_HIP_LIB=rifraf.jl_amd/librifraf_nohalf.so" \
  "RIFRAF_HIP_LIB=rifraf.jl_amd/librifraf_mm1.so" "RIFRAF_HIP_LIB=rifraf.jl_amd/librifraf_noskip.so" || exit 1
mkdir -p gpurun_out/r04g_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_prof/c3 -o p --output-format csv -- python3 scripts/c3_run.py \
  > gpurun_out/r04g_prof/c3.log 2>&1 || { echo "c3 prof failed"; tail -5 gpurun_out/r04g_prof/c3.log; exit 1; }
tail -1 gpurun_out/r04g_prof/c3.log
timeout -k 10 400 python3 scripts/e2e_pinned.py 512 16,1 2,1 2,1,1 2,2 2,2,1 16,2 > gpurun_out/r04g/e2e_pinned.jsonl 2> gpurun_out/r04g/e2e_pinned.err \
  || { echo "e2e pinned failed"; tail -5 gpurun_out/r04g/e2e_pinned.err; exit 1; }
cat gpurun_out/r04g/e2e_pinned.jsonl
