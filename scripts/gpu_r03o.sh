#!/bin/bash
# node-sharded k_agg_loop (in-process ranks, deviceExchange): sharded tests, then the full GPU suite;
# agg-loop breakdown probes on C3 / C4.  Each step time-limited; rc > 1 ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_shagg 600 python -u -m pytest tests/test_gpu_sharded.py -x -v -k "agg_loop or device_exchange" --timeout 150 --timeout-method thread -p no:cacheprovider
step pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step agg_c3 300 python -u scripts/agg_probe.py c3
step agg_c4 300 python -u scripts/agg_probe.py c4
step single_stamps 300 python scripts/single_pod_probe.py stamps
