#!/bin/bash
# helper reordered (staging after the exchange-A pair); C2 with the CPU baseline (chunked spinning pool)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_loop 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "units or prepared or persistent" --timeout 120 --timeout-method thread -p no:cacheprovider
step probe_c2 300 python scripts/c2_host_probe.py stamps
step bench_c2_cpu 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 10
step bench_c1 300 python bench.py --workload c1 --steps 1 --batch 1000 --warmup 1 --cpu-seconds 6
