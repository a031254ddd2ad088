#!/bin/bash
# k_sched_loop: program staging of pod q+2 before (default) or after (libksg_late.so) the helper's granules
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/c2_host_probe.py > gpurun_out/probe_c2.log 2>&1; echo "probe rc=$?"
KSG_LIB=$PWD/kubernetes-kubernetes_amd/lib/libksg_late.so timeout -k 10 300 python scripts/c2_host_probe.py > gpurun_out/probe_c2_late.log 2>&1; echo "probe late rc=$?"
