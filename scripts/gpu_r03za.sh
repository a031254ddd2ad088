#!/bin/bash
# k_agg_loop: the item loop prefetches the next pod's header. Agg tests, agg-workload bench lines.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step agg_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "agg or spill or c3 or c4 or c5"
for w in c3 c4 c4-anti c5 dts; do
  step bench_$w 400 python -u bench.py --workload $w --cpu-seconds 3
done
step c5_growth 500 python -u scripts/c5_growth_probe.py 50
