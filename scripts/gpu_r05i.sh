#!/bin/bash
# round 5: fit kernel phase stamps; gram store-only floor and runtime memset of the same bytes;
# the farm round replayed from a captured graph (tests, c5 lines with / without, kernel trace)
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r05i_fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
LFM_LIBRARY=ablibs/gram/liblfm.so $S r05i_gram_floor 300 python -u scripts/gram_ab.py "" LFM_GRAM_AB=5 MEMSET=1 || exit $?
$S r05i_farm_tests 300 python -u -m pytest tests/test_farm.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
$S r05i_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
LFM_FARM_GRAPH=0 $S r05i_c5_nograph 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
$S r05i_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05i_c5_trace -o run --output-format csv -- \
  python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
echo done
