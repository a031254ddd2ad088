#!/bin/bash
# PodTopologySpread scoring inside k_agg_loop: the targeted tests first, then the agg-loop / parity
# suites, then the DefaultTopologySpreading and C4 bench lines.  Each GPU step has its own time limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_pts 300 python -u -m pytest tests/test_gpu_pts_defaults.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider --maxfail 10
step bench_dts 400 python bench.py --workload dts --steps 3 --warmup 1 --cpu-seconds 5
step bench_c4 400 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 5
