#!/bin/bash
# In-process device-exchange robustness: scripts/shard_probe.py in N fresh processes.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/dx_probe.log
for k in $(seq 1 ${PROBE_RUNS:-6}); do
  timeout -k 10 120 python -u scripts/shard_probe.py ${PROBE_WORLDS:-2d} >> gpurun_out/dx_probe.log 2>&1
  rc=$?; echo "probe $k rc=$rc"; [ $rc -le 1 ] || exit $rc
done
