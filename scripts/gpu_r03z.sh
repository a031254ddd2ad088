#!/bin/bash
# in-process node shards: the re-gate after mid-batch drains (sharded tests, C5 W = 3 probe)
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step shard_tests 500 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread
step shard_c5 400 python -u scripts/shard_probe.py 1,2d,3d c5
