#!/bin/bash
# Round-3 tree on MI355X: full GPU suite + smoke, the loop staging A/B, bench lines for every workload
# (each stream checked against the oracle).  Each step time-limited; rc > 1 ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc
}
step pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step probe_c2 200 python scripts/c2_host_probe.py
KSG_LIB=$PWD/kubernetes-kubernetes_amd/lib/libksg_late.so step probe_c2_late 200 python scripts/c2_host_probe.py
step bench_c2 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 10
step bench_c2_pct0 200 python -u bench.py --steps 5 --warmup 1 --pct 0 --cpu-seconds 3
step bench_c1 200 python -u bench.py --workload c1 --steps 1 --batch 1000 --warmup 1 --cpu-seconds 5
for wl in c3 c4 c4-anti dts c5; do
  step bench_$wl 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-seconds 3
done
