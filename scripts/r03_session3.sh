#!/bin/bash
# PMC passes (scorer issue breakdown, FP64 counters) + e2e profile of the native driver
set -o pipefail
bash scripts/pmc_r03.sh r03pmc || exit 1
mkdir -p gpurun_out/r03e2e
timeout -k 10 300 python scripts/prof_e2e_native.py 1024 > gpurun_out/r03e2e/prof_1024.txt 2>&1 || { echo "e2e prof failed"; tail -20 gpurun_out/r03e2e/prof_1024.txt; exit 1; }
head -5 gpurun_out/r03e2e/prof_1024.txt
