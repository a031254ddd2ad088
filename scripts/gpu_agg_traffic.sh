#!/bin/bash
# k_agg_loop HBM traffic: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes plus a kernel trace,
# each over a short bench run of C3 / C4 / C5 (scripts/prof_summary.py turns them into profiles/).
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for wl in ${WLS:-c4 c5 c3}; do
  B="bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_$wl -o run -- python3 $B > gpurun_out/prof/trace_$wl.log 2>&1
  rc=$?; echo "$wl trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch_$wl -o run -- python3 $B > gpurun_out/prof/fetch_$wl.log 2>&1
  rc=$?; echo "$wl fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write_$wl -o run -- python3 $B > gpurun_out/prof/write_$wl.log 2>&1
  rc=$?; echo "$wl write rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
