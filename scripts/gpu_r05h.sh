#!/bin/bash
# round 5: leading-dimension pads of the gram fill; the fit kernel's phase stamps; a kernel trace
# of the c5 farm round (batch kernel -> ncclAllGather -> publish)
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05h_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
$S r05h_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05h_c5_trace -o run --output-format csv -- \
  python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
echo done
