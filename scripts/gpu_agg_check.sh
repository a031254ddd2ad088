#!/bin/bash
# k_agg_loop: parity tests (random streams vs the launch path and the oracle, C3/C4/C5 streams), then
# bench lines of the aggregation workloads.  Each step time-limited; a crash/timeout ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc
}
step agg_tests 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "agg_loop or c3_ or c4_ or batch_matches or mixed_runs"
step agg_bench_c3 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --cpu-seconds 3
step agg_bench_c4 300 python -u bench.py --workload c4 --steps 2 --warmup 1 --cpu-seconds 3
step agg_bench_c4a 300 python -u bench.py --workload c4-anti --steps 2 --warmup 1 --cpu-seconds 3
step agg_bench_c5 400 python -u bench.py --workload c5 --steps 2 --warmup 1 --cpu-seconds 3
