#!/bin/bash
# k_sched_loop: where the owner workgroup's exchange-A lateness comes from (per-workgroup stamps), C2;
# the CPU baseline's pool scaling on the box's host cores.  Each step time-limited; rc > 1 ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step probe_c2 300 python scripts/c2_host_probe.py
step cpu_pool 300 python scripts/cpu_pool_probe.py
