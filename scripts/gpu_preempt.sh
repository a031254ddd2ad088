#!/bin/bash
# Preemption parity on the GPU box: device golden vectors + random / large-cluster parity.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_preempt.py tests/test_gpu_parity.py -k "preempt or preemption" -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/preempt.log 2>&1
rc=$?; echo "preempt rc=$rc"; exit $rc
