#!/bin/bash
# k_agg_loop without the PodTopologySpread-scoring code for runs that do not score it; resident-loop ring
# changes (single-pod latency); rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the C2 bench.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_agg 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pts_defaults.py tests/test_gpu_sharded.py -x -q -k "agg or c3 or c4 or c5 or default or template or resident" --timeout 150 --timeout-method thread -p no:cacheprovider
step single_pod 300 python scripts/single_pod_probe.py
for wl in c3 c5 c4 dts; do
  step bench_$wl 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 3
done
step prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
step prof_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step prof_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
