#!/bin/bash
# Round 3: tall units split in 64-column halves (default build) against whole (t1) and
# quarter (t4) widths: parity of the default, then the library A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh parity_tall 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_grad.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_tall 500 env AB_ROUNDS=4 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_t1.so dis_project_amd/ab/liblfm_t4.so || exit $?
echo done
