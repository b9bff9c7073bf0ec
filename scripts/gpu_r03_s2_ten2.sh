#!/bin/bash
# Round 3, session 2: the tenancy lock moved into lfm_host.cpp — full -m gpu suite, smoke, and
# the two-ranks-on-one-card rehearsal
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_ten2_suite 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_ten2_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
LFM_BENCH_WATCHDOG=120 scripts/gpu_step.sh s2_ten2_share 200 python -u bench.py --gpus 2 --share-gpus --steps 3 --warmup 1 || exit $?
echo done
