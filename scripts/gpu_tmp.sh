#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "give_up or agg_loop or c3_ or c4_ or c5_ or batch_matches or mixed_runs" > gpurun_out/agg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/agg_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_agg_probe.sh
