#!/bin/bash
# One PMC pass of shader counters (instruction mix, wave cycles, GPU clock) over a short bench run.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/prof/pmc_sq -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; exit $rc
