#!/bin/bash
# Round 3, session 2: tail chain with deferred publication bumps — test, stamps, long A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_tail_test5 300 python -u -m pytest tests/test_gpu_full.py -x -v -k "tail_chain" --timeout 120 --timeout-method thread || exit $?
LFM_TAIL_CHAIN=1 scripts/gpu_step.sh s2_stamps_on5 120 python scripts/chain_stamps.py || exit $?
AB_ROUNDS=12 scripts/gpu_step.sh s2_ab_tail5 500 python -u scripts/ab.py "LFM_TAIL_CHAIN=0" "LFM_TAIL_CHAIN=1" || exit $?
echo done
