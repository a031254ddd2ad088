#!/bin/bash
# sharded device exchange with 128-node loop workgroups + the loopStamps C2 breakdown
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_sharded 400 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider
step probe_c2 300 python scripts/c2_host_probe.py
