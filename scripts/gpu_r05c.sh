#!/bin/bash
# round 5: the c5fit bench line and its kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 > gpurun_out/r05c_c5fit.json 2> gpurun_out/r05c_c5fit.err || { tail -20 gpurun_out/r05c_c5fit.err; exit 2; }
cat gpurun_out/r05c_c5fit.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_prof -o c5fit -- python3 -u bench.py --workload c5fit --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05c_prof.log 2>&1 || { tail -20 gpurun_out/r05c_prof.log; exit 3; }
find gpurun_out/r05c_prof -name "*stats*" | head
