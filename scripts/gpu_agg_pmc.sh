#!/bin/bash
# k_agg_loop shader counters on C4 (two separate passes: SQ issue/wait mix, instruction cache).
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/prof/agg_sq -o run -- python3 scripts/agg_probe.py ${WL:-c4} > gpurun_out/prof/agg_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/prof/agg_ic -o run -- python3 scripts/agg_probe.py ${WL:-c4} > gpurun_out/prof/agg_ic.log 2>&1
rc=$?; echo "ic rc=$rc"; exit $rc
