#!/bin/bash
# One GPU-box pass: sharded tests -> full gpu parity suite -> smoke -> bench lines.  Each GPU step
# has its own time limit; a crash/timeout (rc > 1) ends the script without further GPU work.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step sharded 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 5
step bench_c5 400 python bench.py --workload c5 --steps 2 --warmup 1 --cpu-seconds 10
