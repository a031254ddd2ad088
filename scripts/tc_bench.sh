#!/bin/bash
# k_agg_loop workloads with the template cache on and off (aggLoopDebug 32): one bench line each, no CPU leg
# usage (on the GPU box): scripts/tc_bench.sh <tag> [workloads...]
tag=$1; shift
mkdir -p gpurun_out
for w in "${@:-c3 c5 c4 dts}"; do
  for mode in on off; do
    extra=""; [ $mode = off ] && extra='--extra-config {"aggLoopDebug":32}'
    steps=10; [ $w = c5 ] && steps=20
    timeout -k 10 300 python -u bench.py --workload $w --steps $steps --warmup 1 --no-sub --no-cpu-baseline $extra \
      > gpurun_out/${tag}_${w}_${mode}.json 2> gpurun_out/${tag}_${w}_${mode}.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/${tag}_${w}_${mode}.json').read().strip().splitlines()[-1]); print('$w $mode', d['value'], d['roofline']['avg_kernel_us'], d.get('kernel_us_per_step'))"
  done
done
