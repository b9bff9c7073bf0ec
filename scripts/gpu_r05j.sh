#!/bin/bash
# round 5: the fit kernel's phase stamps (block 0's own history)
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05j_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
echo done
