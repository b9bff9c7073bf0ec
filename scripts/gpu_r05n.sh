#!/bin/bash
# round 5: small kernels with every LDS read of a column / row chunk issued before its first use
# (sched_barrier): tests, fit stamps, c5 and c5fit lines, and a c5 kernel trace
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05n_tests 400 python -u -m pytest tests/test_gpu_batch_grad.py tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05n_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
$S r05n_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
$S r05n_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S r05n_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05n_c5_trace -o run --output-format csv -- \
  python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
echo done
