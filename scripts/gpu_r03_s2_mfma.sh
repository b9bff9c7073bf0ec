#!/bin/bash
# Round 3, session 2: MFMA utilisation by PMC — the production unit alone (step kernel rest role
# over a full T = 127 triangle at depth 640 on the 224 bulk CUs) and every step_kernel dispatch
# of the C2 bench (event-ordered schedule 3, the counters' serialised dispatch)
set -u
export TMPDIR=/tmp PMC_T=127 PMC_KD=640 PMC_CIO=88
mkdir -p gpurun_out
scripts/gpu_step.sh mfma_unit_plain 90 python scripts/pmc_syrk.py 3 || exit $?
scripts/gpu_step.sh mfma_unit 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/mfma_unit -o run --output-format csv -- python3 scripts/pmc_syrk.py 3 || exit $?
LFM_S3_EVENTS=1 scripts/gpu_step.sh mfma_bench 180 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/mfma_bench -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit $?
echo done
