#!/bin/bash
# In-process device-exchange robustness (repeated fresh processes), then the GPU suite and a C2 bench.
# Each GPU step has its own time limit; a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/dx_probe.log
for k in 1 2 3 4 5 6; do
  timeout -k 10 120 python -u scripts/shard_probe.py ${PROBE_WORLDS:-2d} >> gpurun_out/dx_probe.log 2>&1
  rc=$?; echo "probe $k rc=$rc"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
