#!/bin/bash
# Round 3, session 2: rest-triangle supertile size (LFM_SUPERTILE 4 / 6 / 8 / 12): time (A/B)
# and step-kernel PMC bytes per evaluation
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_ab_q 600 python -u scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm_q4.so dis_project_amd/liblfm_q8.so dis_project_amd/liblfm_q12.so || exit $?
bash scripts/pmc_ab.sh liblfm liblfm_q4 liblfm_q8 liblfm_q12 || exit $?
echo done
