#!/bin/bash
# Quick A/B bench: C2 (5 steps), C3, C4 short runs; each step time-limited.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step qb_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 2
step qb_c3 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --cpu-seconds 2
step qb_c4 300 python -u bench.py --workload c4 --steps 2 --warmup 1 --cpu-seconds 2
step qb_c5 400 python -u bench.py --workload c5 --steps 2 --warmup 1 --cpu-seconds 2
