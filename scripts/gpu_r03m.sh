#!/bin/bash
# HEAD check after container re-creation: full GPU suite + smoke, C2 bench with CPU baseline,
# single-pod latency, pct 0, DTS and C3.  Each step time-limited; rc > 1 ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 10
step single_pod 300 python scripts/single_pod_probe.py
step bench_c2_pct0 300 python -u bench.py --steps 5 --warmup 1 --pct 0 --no-cpu-baseline
step bench_c1 300 python -u bench.py --workload c1 --steps 1 --batch 1000 --warmup 1 --cpu-seconds 10
