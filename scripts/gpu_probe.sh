#!/bin/bash
# Loop probe (per-phase stamps, pods/s) then the GPU parity suite; each step time-limited, a crash ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/loop_probe.py ${PROBE_NODES:-5000} ${PROBE_WG:-0} > gpurun_out/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; exit $rc
