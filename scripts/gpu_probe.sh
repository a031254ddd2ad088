export TMPDIR=/tmp
timeout -k 10 200 python scripts/loop_probe.py 5000 20 > gpurun_out/probe.log 2>&1; echo "probe rc=$?"
KSG_LIB=$PWD/kubernetes-kubernetes_amd/lib/libksg_diag.so timeout -k 10 200 python scripts/loop_probe.py 5000 20 >> gpurun_out/probe.log 2>&1; echo "probe-diag rc=$?"
