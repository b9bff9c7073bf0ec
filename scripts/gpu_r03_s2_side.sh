#!/bin/bash
# Round 3, session 2: side-CU partition re-swept on the round-3 kernels (24 / 32 / 40 chain CUs)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=4 scripts/gpu_step.sh s2_ab_side 600 python -u scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm.so@LFM_SIDE_CUS=24 dis_project_amd/liblfm.so@LFM_SIDE_CUS=40 || exit $?
echo done
