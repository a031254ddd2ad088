#!/bin/bash
# GPU parity suite, then one bench line per workload (WLS).  Each GPU step has its own time limit;
# a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
fi
for wl in ${WLS:-c2 c3 c4}; do
  timeout -k 10 400 python bench.py --workload $wl ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"; [ $rc -le 1 ] || exit $rc
done
