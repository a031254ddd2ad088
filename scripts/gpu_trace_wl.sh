#!/bin/bash
# rocprofv3 kernel traces of the launch-path workloads (one short bench run each).
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for wl in ${WLS:-c4 c3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_$wl -o run -- python3 bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_trace_$wl.log 2>&1
  rc=$?; echo "$wl trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
