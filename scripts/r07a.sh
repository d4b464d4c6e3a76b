set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r07a; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "backtrace or bt_ or walk or proposal or frame or workloads" > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
tail -1 $D/tests.log
RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_btwwd4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "backtrace or bt_ or walk or proposal" > $D/tests_wd4.log 2>&1 || { tail -20 $D/tests_wd4.log; exit 1; }
tail -1 $D/tests_wd4.log
for v in hip btwwd4 btwwd6; do
  RIFRAF_HIP_LIB=$PWD/rifraf.jl_amd/librifraf_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/stats_$v -o p --output-format csv -- python3 scripts/c3_run.py > $D/c3_$v.log 2>&1 || { tail -5 $D/c3_$v.log; exit 1; }
  echo "$v done"
done
