#!/bin/bash
# Round 3, session 2: tall units' A21 operand through plain (L2-cached) loads instead of
# device-coherent ones (LFM_TALL_PLAIN_A=1 build): A/B and the full-size parity tests on it
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=5 scripts/gpu_step.sh s2_ab_tpa 500 python -u scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm_tpa.so || exit $?
LFM_LIBRARY=dis_project_amd/liblfm_tpa.so scripts/gpu_step.sh s2_tpa_tests 400 python -u -m pytest tests/test_gpu_full.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread || exit $?
echo done
