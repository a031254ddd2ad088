#!/bin/bash
# PreemptionBasic through ksg_preempt: bench line (1000 and 5000 nodes) + rocprofv3 kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_preempt.py --nodes 1000 --pods 1000 > gpurun_out/preempt_bench_1k.json 2> gpurun_out/preempt_bench_1k.err
rc=$?; echo "bench1k rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_preempt.py --nodes 5000 --pods 1000 --cpu-pods 30 > gpurun_out/preempt_bench_5k.json 2> gpurun_out/preempt_bench_5k.err
rc=$?; echo "bench5k rc=$rc"; [ $rc -le 1 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_preempt -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_preempt.py --nodes 5000 --pods 300 --cpu-pods 1 > $GRAFT_REPO_ROOT/gpurun_out/preempt_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
