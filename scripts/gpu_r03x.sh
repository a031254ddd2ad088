#!/bin/bash
# DF_RAW0 helper fast path: loop parity tests, C2 bench + host probe; C5 batch-by-batch growth probe.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step loop_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "loop or units or prepared or basic or batch or sampling or resident"
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 3
step probe_c2 300 python -u scripts/c2_host_probe.py
step c5_growth 500 python -u scripts/c5_growth_probe.py 50
