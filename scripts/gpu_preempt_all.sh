#!/bin/bash
# Preemption: parity tests, then the PreemptionBasic bench lines and a kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_preempt.py tests/test_gpu_parity.py -k "preempt or preemption" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/preempt.log 2>&1
rc=$?; echo "preempt tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_preempt_bench.sh
