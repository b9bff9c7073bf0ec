#!/bin/bash
# round 5: the two-lanes-per-row sweep (n + 1 <= 32): batch-gradient tests twice, the farm /
# parity / edge tests, fit stamps, the c5fit line, the fit diagnostic
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05u_tests_a 300 python -u -m pytest tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S r05u_tests_b 300 python -u -m pytest tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S r05u_tests 400 python -u -m pytest tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05u_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
$S r05u_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S r05u_diag 200 python -u scripts/diag_fit.py || exit $?
echo done
