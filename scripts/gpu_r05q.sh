#!/bin/bash
# round 5: flattened grid reduction of the small gradient; the batch-gradient tests twice (a
# mismatch seen once on r05n's box), the rest of the small-kernel tests, stamps, c5 / c5fit lines
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05q_tests_a 300 python -u -m pytest tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S r05q_tests_b 300 python -u -m pytest tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S r05q_tests 400 python -u -m pytest tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05q_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
$S r05q_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
$S r05q_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S r05q_diag 200 python -u scripts/diag_fit.py || exit $?
echo done
