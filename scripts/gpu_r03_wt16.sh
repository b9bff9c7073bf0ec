#!/bin/bash
# Round 3: 16-B write-through C tiles (default) against 8-B (wt8): parity, library A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh parity_wt16 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_grad.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_wt16 400 env AB_ROUNDS=5 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_wt8.so || exit $?
scripts/gpu_step.sh grad_wt16 200 python scripts/grad_time.py || exit $?
echo done
