#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (the roofline kernel's average duration
# must agree with bench.py's live HIP-event figure), then a separate PMC pass for HBM bytes.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof/bench_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof/bench_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; exit $rc
