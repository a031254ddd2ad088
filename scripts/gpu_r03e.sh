#!/bin/bash
# k_sched_loop with exchange A carried inside exchange B: loop parity, sharded, C2 bench + loopStamps
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_loop 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "units or prepared or persistent or ties or basic or batch" --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_sharded 400 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_c2 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step probe_c2 300 python scripts/c2_host_probe.py
