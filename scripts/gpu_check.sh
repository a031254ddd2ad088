#!/bin/bash
# One GPU-box pass: smoke -> gpu parity tests -> short bench.  Each GPU step has its own time
# limit; a crash/timeout (rc > 1) ends the script without starting further GPU work.
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --cpu-seconds 5"}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=${MAXFAIL:-40} -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
