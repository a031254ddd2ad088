#!/bin/bash
# Loop change check: loop/stream parity tests -> loop probe (per-phase stamps) -> C2 bench.
# Each GPU step is time-limited; a crash/timeout (rc > 1) ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step loop_tests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${KSEL:-loop or basic or pipeline or sampling or stream or random or batch}"
step probe 200 python -u scripts/loop_probe.py 5000 0
step bench_c2 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 3
