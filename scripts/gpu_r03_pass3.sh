#!/bin/bash
# Round 3, third pass: the -m gpu suite on the final kernel, and the library A/B against the
# round-2 build (dis_project_amd/ab/liblfm_r02.so, built from commit 055b4e0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_lib_r02 400 env AB_ROUNDS=4 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_r02.so || exit $?
echo done
