#!/bin/bash
# sharded tests + the W = 3 pipelined diagnostic; rocprofv3 kernel trace + FETCH / WRITE passes of C2;
# FETCH / WRITE passes of C4-anti and DefaultTopologySpreading (k_agg_loop traffic).
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step shard_tests 500 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step w3_probe 200 python -u scripts/w3_pipelined_probe.py 3 2
step prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step prof_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
for wl in c4-anti dts; do
  B="bench.py --workload $wl --steps 1 --warmup 1 --no-cpu-baseline"
  step trace_$wl 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_$wl -o run -- python3 $B
  step fetch_$wl 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch_$wl -o run -- python3 $B
  step write_$wl 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write_$wl -o run -- python3 $B
done
