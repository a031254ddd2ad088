#!/bin/bash
# k_agg_loop HBM spill rows: agg parity tests, the C5 batch-by-batch probe, the C5 bench at 50 000 pods.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step agg_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "agg or spill"
step c5_growth 500 python -u scripts/c5_growth_probe.py 50
step bench_c5_50k 600 python -u bench.py --workload c5 --steps 50 --warmup 1 --cpu-seconds 10
