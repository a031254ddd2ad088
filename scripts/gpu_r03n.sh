#!/bin/bash
# percentageOfNodesToScore inside k_sched_loop: sampling parity (loop, batch, resident), pct 0 / 100 bench,
# single-pod latency.  Each step time-limited; rc > 1 ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_samp 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sampling or resident or units or prepared" --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_c2_pct0 300 python -u bench.py --steps 10 --warmup 2 --pct 0 --no-cpu-baseline
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
step single_pod 300 python scripts/single_pod_probe.py
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
