#!/bin/bash
# Round 3, session 2: quarter-width tall units (LFM_TALL_SPLIT=4 build) against the default
# (2) now that the tall units are dealt round-robin to the XCDs: A/B, then the full-size tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_ROUNDS=6 scripts/gpu_step.sh s2_ab_ts4 500 python -u scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/liblfm_ts4.so || exit $?
LFM_LIBRARY=dis_project_amd/liblfm_ts4.so scripts/gpu_step.sh s2_ts4_tests 400 python -u -m pytest tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread || exit $?
echo done
