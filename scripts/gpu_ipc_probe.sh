#!/bin/bash
# Two processes on the box's GPU: the server polls granules the client stores over IPC (scripts/ipc_probe.hip).
export TMPDIR=/tmp
mkdir -p gpurun_out
f=/tmp/ipc_handle_$$
rm -f $f
timeout -k 5 60 scripts/ipc_probe server $f > gpurun_out/ipc_server.log 2>&1 &
sp=$!
timeout -k 5 60 scripts/ipc_probe client $f > gpurun_out/ipc_client.log 2>&1
crc=$?
wait $sp
src=$?
echo "ipc client rc=$crc server rc=$src"
[ $crc -eq 0 ] && [ $src -eq 0 ]
