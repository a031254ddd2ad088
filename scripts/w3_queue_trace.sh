#!/bin/bash
# The W = 3 in-process k_agg_loop test under rocprofv3 --kernel-trace, to record which hardware queue each
# rank's loop dispatch went to (the round-4 give-up's cause).  Run on the GPU box:
#   gpurun -- bash scripts/w3_queue_trace.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for k in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/w3q_$k -o run -- \
    python3 -m pytest -x -q -p no:cacheprovider tests/test_gpu_sharded.py -m gpu \
    -k "c5_pipelined_batches_sharded_agg_loop and 3" > gpurun_out/w3q_$k.log 2>&1 || exit $?
  tail -2 gpurun_out/w3q_$k.log
done
