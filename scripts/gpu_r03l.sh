#!/bin/bash
# resident single-pod loop: call breakdown, latency; batch k_sched_loop back to its own instance (C2)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_resident 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "resident or units" --timeout 120 --timeout-method thread -p no:cacheprovider
step single_pod_stamps 300 python scripts/single_pod_probe.py stamps
step single_pod 300 python scripts/single_pod_probe.py
step bench_c2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline
