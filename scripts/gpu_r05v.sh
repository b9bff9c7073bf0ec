#!/bin/bash
# round 5: the small kernels' Qt table entries without their erfcx term (a per-gene entry):
# tests, both stamps, c5 / c5fit lines
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05v_tests 400 python -u -m pytest tests/test_gpu_batch_grad.py tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05v_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
LFM_LIBRARY=ablibs/stamps/liblfm.so $S r05v_small_stamps 120 python -u scripts/small_stamps.py || exit $?
$S r05v_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
$S r05v_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
echo done
