#!/bin/bash
# k_sched_loop helper with hoisted LDS reads; k_agg_loop DF_AGG_SAME (no gather for same-template pods):
# loop parity tests, C2 / C4 / C4-anti / DTS benches with the oracle check, C2 owner probe, full suite.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_loops 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pts_defaults.py -x -q -k "loop or agg or units or prepared or basic or batch or c3 or c4 or c5 or default or template" --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 3
step bench_c4 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 3
step bench_c4a 300 python -u bench.py --workload c4-anti --steps 3 --warmup 1 --cpu-seconds 3
step bench_dts 300 python -u bench.py --workload dts --steps 3 --warmup 1 --cpu-seconds 3
step probe_c2 300 python scripts/c2_host_probe.py
step pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
