#!/bin/bash
# GPU-box runner: each step under its own time limit; a step that faults,
# aborts or times out (any exit status other than 0 / 1) ends the script.
# Usage: tools/gpu_run.sh NAME SECONDS CMD... [--- NAME SECONDS CMD...]...
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
    name=$1; secs=$2; shift 2
    cmd=()
    while [ $# -gt 0 ] && [ "$1" != "---" ]; do cmd+=("$1"); shift; done
    [ "$1" = "---" ] && shift
    echo "[gpu_run] $name: ${cmd[*]}"
    timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
    rc=$?
    tail -3 "gpurun_out/$name.log"
    echo "[gpu_run] $name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_run] stopping after $name"; exit $rc; fi
done
