#!/bin/bash
# resident single-pod loop: parity (single calls with stops / relaunches), latency probe; loop batch parity + C2
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_resident 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "resident" --timeout 120 --timeout-method thread -p no:cacheprovider
step single_pod 300 python scripts/single_pod_probe.py
step pytest_loop 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "units or prepared or persistent or basic or batch or random" --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_c2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
