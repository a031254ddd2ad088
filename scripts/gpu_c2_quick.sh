#!/bin/bash
# C2 A/B: bench line (parity-checked) and the host probe.  Each GPU step has its own time limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step bench_c2 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 3
step host_probe 300 python -u scripts/c2_host_probe.py
