#!/bin/bash
# preemption (self-affinity on the device) + the full GPU suite
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_preempt 400 python -u -m pytest tests/test_gpu_preempt.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider
step pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
