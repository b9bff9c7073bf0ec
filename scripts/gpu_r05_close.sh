#!/bin/bash
# Round 5's closing measurements on the final library (GPU box, repo root): the default bench line
# (C2), the C5 and C5-fit lines, a C5 kernel trace, the MLL kernel's phase stamps and clock, the
# -m gpu suite and smoke(). Every step under its own time limit (scripts/gpu_step.sh); the first
# failure ends the run.
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S close_c2 600 python -u bench.py || exit $?
$S close_c5 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 || exit $?
$S close_c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S close_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/close_c5_trace -o run \
  --output-format csv -- python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
LFM_LIBRARY=ablibs/stamps/liblfm.so $S close_stamps 120 python -u scripts/small_stamps.py || exit $?
$S close_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
$S close_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
echo done
