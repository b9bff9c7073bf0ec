#!/bin/bash
# Round 3, session 2: the final tree — full -m gpu suite, smoke, the default bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_end_suite 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_end_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
scripts/gpu_step.sh s2_end_bench 300 python bench.py || exit $?
echo done
