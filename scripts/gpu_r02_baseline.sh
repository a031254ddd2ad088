#!/bin/bash
# Round-2 baseline: bench lines for every workload, then rocprofv3 kernel traces of C3/C4/C5.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash scripts/gpu_bench_all.sh || exit $?
WLS="c3 c4 c5" bash scripts/gpu_trace_wl.sh || exit $?
