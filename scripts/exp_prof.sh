#!/bin/bash
# Per-kernel times of experimental builds: scripts/exp_prof.sh NAME... (librifraf_NAME.so;
# "hip" = the product library).  Output: gpurun_out/expprof/NAME/k_kernel_stats.csv + summary.
export TMPDIR=/tmp
mkdir -p gpurun_out/expprof
for v in "$@"; do
  export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so
  [ "$v" = hip ] && export RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_hip.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/expprof/$v -o k --output-format csv -- \
    python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/expprof/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/expprof/$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/expprof/{v}/k_kernel_stats.csv")))
print(v, "  ".join(f"{r['Name'].split('(')[0].replace('void ','')}={float(r['AverageNs'])/1e6:.2f}ms" for r in rows if float(r['Percentage']) > 1.0))
PY
done
