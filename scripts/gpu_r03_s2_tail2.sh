#!/bin/bash
# Round 3, session 2: persistent tail chain — the rest of the suite after the forced-helper fix,
# the interleaved A/B and the step timeline
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_tail_suite 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
AB_ROUNDS=8 scripts/gpu_step.sh s2_ab_tail 300 python -u scripts/ab.py "LFM_TAIL_CHAIN=0" "LFM_TAIL_CHAIN=1" || exit $?
scripts/gpu_step.sh s2_tail_timeline 200 python scripts/step_timeline.py --json gpurun_out/s2_tail_timeline.json || exit $?
echo done
