#!/bin/bash
# Full GPU parity suite, then the single-pod latency probe.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/single_pod_probe.py > gpurun_out/single.json 2> gpurun_out/single.err
rc=$?; echo "single rc=$rc"; exit $rc
