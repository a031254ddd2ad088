#!/bin/bash
# Round-3 first pass: the new default-constraint / boundary tests and the golden vectors on the device,
# the whole GPU suite, then the C2 and DefaultTopologySpreading bench lines.  Each GPU step has its own
# time limit; a crash / timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_new 400 python -u -m pytest tests/test_gpu_pts_defaults.py tests/test_gpu_boundary.py -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider --maxfail 20
step bench_c2 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5
step bench_dts 400 python bench.py --workload dts --steps 3 --warmup 1 --cpu-seconds 5
