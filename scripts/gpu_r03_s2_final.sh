#!/bin/bash
# Round 3, session 2: the full -m gpu suite on the final code (incl. the full-size tenancy
# regression test) and smoke
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_final_suite 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_final_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
echo done
