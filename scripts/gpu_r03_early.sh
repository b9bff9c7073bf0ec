#!/bin/bash
# Round 3: early units (LFM_EARLY) — bit-identity tests, interleaved A/B of the region size and
# of the step widths it applies to, and the step timeline with them on.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh early_tests 600 python -u -m pytest tests/test_gpu_full.py -m gpu -x -v -k early --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_early 400 env AB_ROUNDS=6 python scripts/ab.py "LFM_EARLY=0" "LFM_EARLY=30" "LFM_EARLY=18" "LFM_EARLY=42" "LFM_EARLY=30 LFM_EARLY_WMIN=1" "LFM_EARLY=12 LFM_EARLY_WMIN=1" || exit $?
scripts/gpu_step.sh tl_early 180 env LFM_EARLY=30 python scripts/step_timeline.py --json gpurun_out/r03_tl_early30.json || exit $?
scripts/gpu_step.sh tl_base 180 env LFM_EARLY=0 python scripts/step_timeline.py --json gpurun_out/r03_tl_early0.json || exit $?
echo done
