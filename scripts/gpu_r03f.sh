#!/bin/bash
# diagnostic build: k_sched_loop phase-1 / eval_core_fast step stamps at C2
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
KSG_LIB=$PWD/kubernetes-kubernetes_amd/lib/libksg_diag.so step probe_diag 300 python scripts/c2_host_probe.py stamps
step bench_c2_cpu 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 10
step bench_c1 300 python bench.py --workload c1 --steps 1 --batch 1000 --warmup 1 --cpu-seconds 6
