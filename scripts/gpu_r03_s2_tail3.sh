#!/bin/bash
# Round 3, session 2: tail chain knobs (start size LFM_TAIL_M, poll nap LFM_TAIL_NAP), its test
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_tail_test3 300 python -u -m pytest tests/test_gpu_full.py -x -v -k "tail_chain" --timeout 120 --timeout-method thread || exit $?
AB_ROUNDS=8 scripts/gpu_step.sh s2_ab_tail3 500 python -u scripts/ab.py "LFM_TAIL_CHAIN=0" "LFM_TAIL_CHAIN=1" "LFM_TAIL_CHAIN=1 LFM_TAIL_NAP=1" "LFM_TAIL_CHAIN=1 LFM_TAIL_M=3584" "LFM_TAIL_CHAIN=1 LFM_TAIL_M=3584 LFM_TAIL_NAP=1" "LFM_TAIL_CHAIN=1 LFM_TAIL_M=2560 LFM_TAIL_NAP=1" || exit $?
echo done
