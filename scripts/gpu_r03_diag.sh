#!/bin/bash
# diagnostic build: k_sched_loop phase-1 section stamps (C2), via the c2 host probe's loopStamps batch
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
KSG_LIB=kubernetes-kubernetes_amd/lib/libksg_diag.so step diag_c2 300 python -u scripts/c2_host_probe.py
