#!/bin/bash
# C5 at BASELINE's 50 000 measured pods; in-process node-sharded loops (W = 1, 2, 3) on C4 / C5 with the
# device exchange (k_agg_loop<true>) and with the all-reduce path.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step bench_c5_50k 600 python -u bench.py --workload c5 --steps 50 --warmup 1 --cpu-seconds 10
step shard_c4 300 python -u scripts/shard_probe.py 1,2d,2r,3d c4
step shard_c5 400 python -u scripts/shard_probe.py 1,2d,2r,3d c5
