#!/bin/bash
# Full GPU parity suite + smoke, then bench lines for C2..C5.  Each GPU step has its own time limit;
# a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5
for wl in c3 c4 c4-anti c5; do
  step bench_$wl 400 python bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 5
done
