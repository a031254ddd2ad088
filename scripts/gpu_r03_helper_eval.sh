#!/bin/bash
# k_sched_loop (128-node units): the helper evaluates its candidate with the pod assumed; phase 1 evaluates
# each node once. Loop parity tests, C1 / C2 / pct-0 bench lines, the C2 host probe.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step loop_tests 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "loop or units or prepared or basic or batch or sampling or resident or sharded or smoke"
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 3
step bench_c1 300 python -u bench.py --workload c1 --steps 10 --warmup 2 --cpu-seconds 3
step bench_c2_pct0 300 python -u bench.py --steps 10 --warmup 2 --pct 0 --cpu-seconds 3
step probe_c2 300 python -u scripts/c2_host_probe.py
