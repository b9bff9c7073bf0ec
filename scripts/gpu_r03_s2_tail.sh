#!/bin/bash
# Round 3, session 2: persistent tail chain (LFM_TAIL_CHAIN) — its test, the parity suites
# that cover the tail, the interleaved A/B and the step timeline
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_tail_test 300 python -u -m pytest tests/test_gpu_full.py -x -v -k "tail_chain" --timeout 120 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_tail_parity 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_regimes.py -x -q --timeout 200 --timeout-method thread || exit $?
AB_ROUNDS=8 scripts/gpu_step.sh s2_ab_tail 300 python -u scripts/ab.py "LFM_TAIL_CHAIN=0" "LFM_TAIL_CHAIN=1" || exit $?
scripts/gpu_step.sh s2_tail_timeline 200 python scripts/step_timeline.py --json gpurun_out/s2_tail_timeline.json || exit $?
echo done
