#!/bin/bash
# Full GPU parity suite, then bench lines for the aggregation workloads and the C3 phase probe.
# Each GPU step has its own time limit; a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for wl in c3 c4 c4-anti c5; do
  step bench_$wl 400 python bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 5
done
step agg_probe_c3 300 python -u scripts/agg_probe.py c3
