#!/bin/bash
# Round 3: trailing-update tile body on v_mfma_f64_16x16x4_f64 (default build) against the
# 4x4x4_4b body (dis_project_amd/ab/liblfm_m4.so, -DLFM_MFMA16=0): library A/B, then parity
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh ab_m16 400 env AB_ROUNDS=4 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_m4.so || exit $?
scripts/gpu_step.sh parity_m16 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
echo done
