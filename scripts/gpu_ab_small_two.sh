#!/bin/bash
# The MLL factor's two-lane LDL^T columns (LFM_SMALL_TWO, default) against ablibs/notwo
# (make EXTRA=-DLFM_SMALL_TWO=0): the small-kernel GPU tests, block 0's phase stamps, C5 lines
# interleaved (r05_ab_small_two.txt)
set -u
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S two_tests 600 python -u -m pytest tests/test_farm.py tests/test_gpu_parity.py tests/test_gpu_edges.py \
  tests/test_gpu_regimes.py tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/stamps/liblfm.so $S two_stamps 120 python -u scripts/small_stamps.py || exit $?
for i in 1 2 3; do
  $S two_on_$i 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
  LFM_LIBRARY=ablibs/notwo/liblfm.so $S two_off_$i 300 python -u bench.py --workload c5 --steps 3000 \
    --warmup 300 --no-cpu-baseline || exit $?
done
echo done
