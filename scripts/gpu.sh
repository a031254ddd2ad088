#!/bin/bash
# The one GPU-box runner (replaces the per-round scripts/gpu_*.sh one-offs).
#
#   gpurun -- bash scripts/gpu.sh STEP [STEP ...]
#
# Steps (each GPU step has its own time limit; a crash, abort or timeout (rc > 1) ends the script
# before any further GPU work; every step writes gpurun_out/<name>.log):
#   suite               pytest -m gpu, whole suite
#   tests=<file[::k]>   pytest on one file / node id (-m gpu)
#   smoke               __graft_entry__.smoke()
#   benchdefault        bench.py with no arguments, as the driver runs it (C2 + the C5 100k sub-record)
#   bench=<wl>[:steps]  bench.py --workload <wl> (c1 c2 c2pct0 c3 c4 c4-anti c5 dts), 3 steps by default
#   prof=<wl>           rocprofv3 --kernel-trace --stats of a short bench run of <wl>
#   pmc=<wl>            FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 runs) of <wl>
#   sq=<wl>             one shader-counter pass (instruction mix, wave cycles, clock) of <wl>
#   py=<script>[:args]  python3 -u scripts/<script> args (probes); ',' in args becomes ' '
#   repeat=<n>:<script>[:args]  the probe in n fresh processes (e.g. the in-process device-exchange start)
#   pydiag=<script>[:args]  as py=, on the diagnostic library (make -C kubernetes-kubernetes_amd diag; KSG_LIB)
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ $rc -le 1 ] || exit $rc
}
bench_args() {  # workload -> bench.py arguments
  case $1 in
    c2pct0) echo "--workload c2 --pct 0" ;;
    c1solo) echo "--workload c1 --extra-config {\"loopWorkgroups\":1,\"loopUnit\":256}" ;;
    c1g2) echo "--workload c1 --extra-config {\"loopWorkgroups\":2,\"loopUnit\":256}" ;;
    *) echo "--workload $1" ;;
  esac
}
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    suite) step suite 900 $PYT tests -m gpu ;;
    tests=*) f=${s#tests=}; n=$(basename "$f"); n=${n//[^A-Za-z0-9]/_}; step "tests_${n:0:80}" 600 $PYT "$f" -m gpu -v ;;
    smoke) step smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    benchdefault) step bench_default 600 python -u bench.py ;;
    bench=*)
      a=${s#bench=}; wl=${a%%:*}; n=3; [ "$a" != "$wl" ] && n=${a#*:}
      step "bench_$wl" 400 python -u bench.py $(bench_args "$wl") --steps "$n" --warmup 1 --cpu-seconds 5 ;;
    prof=*)
      wl=${s#prof=}
      export KSG_LOOP_PODS_OUT="gpurun_out/prof/loop_pods_trace_$wl.json"
      step "prof_$wl" 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof/trace_$wl" -o run -- \
        python3 bench.py $(bench_args "$wl") --steps 3 --warmup 1 --no-cpu-baseline --no-sub
      unset KSG_LOOP_PODS_OUT ;;
    pmc=*)
      wl=${s#pmc=}
      # (each pass also writes the pods every loop kernel ran: bench.py KSG_LOOP_PODS_OUT)
      export KSG_LOOP_PODS_OUT="gpurun_out/prof/loop_pods_fetch_$wl.json"
      step "pmcf_$wl" 300 rocprofv3 --pmc FETCH_SIZE -d "gpurun_out/prof/pmc_fetch_$wl" -o run -- \
        python3 bench.py $(bench_args "$wl") --steps 1 --warmup 1 --no-cpu-baseline --no-sub
      export KSG_LOOP_PODS_OUT="gpurun_out/prof/loop_pods_write_$wl.json"
      step "pmcw_$wl" 300 rocprofv3 --pmc WRITE_SIZE -d "gpurun_out/prof/pmc_write_$wl" -o run -- \
        python3 bench.py $(bench_args "$wl") --steps 1 --warmup 1 --no-cpu-baseline --no-sub
      unset KSG_LOOP_PODS_OUT ;;
    sq=*)
      wl=${s#sq=}
      step "sq_$wl" 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        GRBM_GUI_ACTIVE GRBM_COUNT -d "gpurun_out/prof/pmc_sq_$wl" -o run -- \
        python3 bench.py $(bench_args "$wl") --steps 1 --warmup 1 --no-cpu-baseline ;;
    repeat=*)
      a=${s#repeat=}; n=${a%%:*}; rest=${a#*:}; sc=${rest%%:*}; args=""; [ "$rest" != "$sc" ] && args=${rest#*:}
      for k in $(seq 1 "$n"); do step "repeat_${sc%.py}_$k" 200 python3 -u "scripts/$sc" ${args//,/ }; done ;;
    pydiag=*)
      a=${s#pydiag=}; sc=${a%%:*}; args=""; [ "$a" != "$sc" ] && args=${a#*:}
      n=${args//[^A-Za-z0-9]/_}; step "pydiag_${sc%.py}${n:+_${n:0:40}}" 400 env KSG_LIB="$PWD/kubernetes-kubernetes_amd/lib/libksg_diag.so" python3 -u "scripts/$sc" ${args//,/ } ;;
    py=*)
      a=${s#py=}; sc=${a%%:*}; args=""; [ "$a" != "$sc" ] && args=${a#*:}
      n=${args//[^A-Za-z0-9]/_}; step "py_${sc%.py}${n:+_${n:0:40}}" 400 python3 -u "scripts/$sc" ${args//,/ } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
