#!/bin/bash
# Bench lines for every workload (c2 default, c2-hetero, c3, c4, c4-anti, c5); each step time-limited,
# a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step bench_c2 300 python -u bench.py
step bench_c2h 300 python -u bench.py --workload c2-hetero --steps 5 --warmup 1 --cpu-seconds 5
step bench_c3 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --cpu-seconds 5
step bench_c4 300 python -u bench.py --workload c4 --steps 2 --warmup 1 --cpu-seconds 5
step bench_c4a 300 python -u bench.py --workload c4-anti --steps 2 --warmup 1 --cpu-seconds 5
step bench_c5 400 python -u bench.py --workload c5 --steps 2 --warmup 1 --cpu-seconds 10
