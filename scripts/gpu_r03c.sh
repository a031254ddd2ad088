#!/bin/bash
# k_sched_loop with 128-node workgroups: parity (new unit test, the loop / sharded suites), then C2 bench
# lines for both units and a loopStamps breakdown.  Each GPU step has its own time limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_unit 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "units or persistent or ties or basic or batch" --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider --maxfail 10
step bench_c2 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 3
step bench_c2_u256 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra-config '{"loopUnit": 256}'
step probe_c2 300 python scripts/c2_host_probe.py
