#!/bin/bash
# Loop check + two PMC passes over a short C2 bench (instruction issue / wait mix; instruction cache).
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step loop_tests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${KSEL:-loop or basic or pipeline or sampling or stream or random or batch}"
step probe 200 python -u scripts/loop_probe.py 5000 0
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH -d gpurun_out/prof/pmc_sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_ic 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/prof/pmc_ic -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
