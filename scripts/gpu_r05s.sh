#!/bin/bash
# round 5: the gradient's W rows at compile-time offsets; tests, fit stamps, c5 / c5fit lines,
# the MLL kernel's phase stamps (ablibs/stamps) and a c5 kernel trace
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05s_tests 400 python -u -m pytest tests/test_gpu_batch_grad.py tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05s_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
LFM_LIBRARY=ablibs/stamps/liblfm.so $S r05s_small_stamps 120 python -u scripts/small_stamps.py || exit $?
$S r05s_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
$S r05s_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S r05s_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s_c5_trace -o run --output-format csv -- \
  python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
echo done
