#!/bin/bash
# Round-3 final tree: full GPU parity suite + smoke, then every bench line (parity-checked).
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5
step bench_c1 300 python -u bench.py --workload c1 --steps 10 --warmup 2 --cpu-seconds 3
step bench_c2_pct0 300 python -u bench.py --steps 10 --warmup 2 --pct 0 --cpu-seconds 3
for wl in c3 c4 c4-anti c5 dts; do
  step bench_$wl 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 3
done
