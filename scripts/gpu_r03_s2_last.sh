#!/bin/bash
# Round 3, session 2, last pass on the final tree: full -m gpu suite (incl. the edge-input
# tests), smoke, and the default bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_last_suite 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_last_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
scripts/gpu_step.sh s2_last_bench 300 python -u bench.py || exit $?
echo done
