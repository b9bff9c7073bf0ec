#!/bin/bash
# Round 3, session 2: tail chain, late starts only, and chain stamps with / without it
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=8 scripts/gpu_step.sh s2_ab_tail4 400 python -u scripts/ab.py "LFM_TAIL_CHAIN=0" "LFM_TAIL_CHAIN=1 LFM_TAIL_M=2048" "LFM_TAIL_CHAIN=1 LFM_TAIL_M=1024" "LFM_TAIL_CHAIN=1" || exit $?
LFM_TAIL_CHAIN=0 scripts/gpu_step.sh s2_stamps_off 120 python scripts/chain_stamps.py || exit $?
LFM_TAIL_CHAIN=1 scripts/gpu_step.sh s2_stamps_on 120 python scripts/chain_stamps.py || exit $?
echo done
