#!/bin/bash
# Round 3, session 2: the tenancy tests (after the regression test's output fix) and smoke
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_final_tenancy 300 python -u -m pytest tests/test_gpu_tenancy.py -x -v --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_final_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
echo done
