#!/bin/bash
# bench lines of the final round-3 tree (every BASELINE workload, parity-checked), C5 at 50 000 pods
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5
step bench_c2_pct0 300 python -u bench.py --steps 10 --warmup 2 --pct 0 --cpu-seconds 3
for wl in c3 c4 c4-anti c5 dts; do
  step bench_$wl 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 3
done
step bench_c5_50k 600 python -u bench.py --workload c5 --steps 50 --warmup 1 --cpu-seconds 5
