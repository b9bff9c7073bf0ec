#!/bin/bash
# Round 3: tall units round-robin over the XCDs (default) against contiguous ranges (rr0) and
# round-robin half-width pieces (t2): parity of the default, library A/B, a unit trace
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh parity_rr 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full.py tests/test_gpu_grad.py -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_rr 500 env AB_ROUNDS=4 python scripts/ab_lib.py dis_project_amd/liblfm.so dis_project_amd/ab/liblfm_rr0.so dis_project_amd/ab/liblfm_t2.so || exit $?
scripts/gpu_step.sh trace_rr 200 python -u scripts/unit_trace.py gpurun_out/unit_trace_rr.npz || exit $?
echo done
