#!/bin/bash
# k_sched_loop wave-role maps: parity tests for maps 1 and 2, then the C2 probe over maps 0..2.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step wavemap_tests 300 python -u -m pytest tests/test_gpu_parity.py -k "wave_maps or loop_geometries or mixed_runs" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
step wavemap_probe 400 python -u scripts/c2_host_probe.py wavemap
