#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "gather or churn or forget or node_updates or give_up or agg_loop or batch_matches or mixed_runs or c3_pod or c4_topology" > gpurun_out/agg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/agg_tests.log; exit $rc
