#!/bin/bash
# Run one named GPU step under its own time limit, log to gpurun_out/<name>.log and
# record the exit status. Usage: scripts/gpu_step.sh NAME SECONDS CMD...
# Exit status: the command's. Callers chain steps with && and stop on the first
# crash-class status (124/134/137/139) — never retry a GPU step.
set -u
name=$1; to=$2; shift 2
mkdir -p gpurun_out
start=$(date +%s)
timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "$name rc=$rc $(( $(date +%s) - start ))s" >> gpurun_out/steps.log
tail -n 5 "gpurun_out/$name.log"
exit $rc
