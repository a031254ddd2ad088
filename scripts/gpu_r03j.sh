#!/bin/bash
# the oracle CPU baseline's pool settings on the GPU box's host cores (no GPU work)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step cpu_crash 300 python -X faulthandler scripts/pw_crash_probe.py
step cpu_pool 400 python -X faulthandler scripts/cpu_pool_probe.py
