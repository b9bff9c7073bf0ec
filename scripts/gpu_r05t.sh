#!/bin/bash
# round 5: the full GPU suite and the smoke test on the current library
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
$S r05t_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S r05t_suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
echo done
