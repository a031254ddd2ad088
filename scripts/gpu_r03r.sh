#!/bin/bash
# k_sched_loop owner probe (last evaluation wave's phase-1 end)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/c2_host_probe.py > gpurun_out/probe_c2.log 2>&1; echo "probe rc=$?"
