#!/bin/bash
# Round 3, session 2: readers-writer device tenancy (tests + two ranks on one card through the
# RCCL-failure fallback), then the first-super-panel width A/B (LFM_W0)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_tenancy 300 python -u -m pytest tests/test_gpu_tenancy.py -x -v --timeout 120 --timeout-method thread || exit $?
LFM_BENCH_WATCHDOG=100 scripts/gpu_step.sh s2_rccl_share3 160 python -u bench.py --gpus 2 --share-gpus --steps 3 --warmup 1 || exit $?
AB_ROUNDS=6 scripts/gpu_step.sh s2_ab_w0 300 python -u scripts/ab.py "LFM_W0=1" "LFM_W0=2" || exit $?
echo done
