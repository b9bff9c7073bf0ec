#!/bin/bash
# round 5: the sweep-operator gradient path (one wave): batch gradient / fit tests, fit stamps,
# the c5fit line
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05k_tests 400 python -u -m pytest tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05k_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
$S r05k_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
echo done
