#!/bin/bash
# scalar check decided at decode: full GPU suite, smoke, default + C1 bench lines, C2 host probe
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python -u bench.py
step bench_c1 300 python -u bench.py --workload c1 --cpu-seconds 3
step probe_c2 300 python -u scripts/c2_host_probe.py
