#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread \
  -k "give_up or agg_loop or c3_ or c4_ or c5_ or batch_matches or mixed_runs or persistent_loop or pipeline or basic or ties or device_exchange" > gpurun_out/agg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/agg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 2 > gpurun_out/bench_c2.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_c2.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
WLS="c4 c3" bash scripts/gpu_agg_probe.sh
