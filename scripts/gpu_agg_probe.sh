#!/bin/bash
# k_agg_loop phase breakdown (loopStamps) on C3 / C4 / C4-anti / C5.
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in ${WLS:-c3 c4 c4-anti c5}; do
  timeout -k 10 300 python -u scripts/agg_probe.py $wl > gpurun_out/agg_probe_$wl.log 2>&1
  rc=$?; echo "$wl rc=$rc"; grep -E "k_agg_loop (stamps|skew|phase 2)|pods/s" gpurun_out/agg_probe_$wl.log; [ $rc -eq 0 ] || exit $rc
done
