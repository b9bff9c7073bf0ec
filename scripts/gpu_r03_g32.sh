#!/bin/bash
# Round 3: the chain's gemm32 on 16x16x4 (default) against 4x4x4 (g0); settings sweep of the
# plan and the side-CU helper on the current kernels; parity of the default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh parity_g32 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_grad.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_g32 400 env AB_ROUNDS=4 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_g0.so || exit $?
scripts/gpu_step.sh ab_knobs 500 env AB_ROUNDS=6 python scripts/ab.py "" "LFM_HELPER_TC=600" "LFM_HELPER_TC=800" "LFM_HELPER_MIN=800" "LFM_HELPER_MIN=1600" "LFM_W4_MIN=5120" "LFM_W4_MIN=7168" "LFM_W2_MIN=4608" "LFM_W2_MIN=5632" || exit $?
echo done
