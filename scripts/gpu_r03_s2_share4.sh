#!/bin/bash
# Round 3, session 2: the N = 4 rank path rehearsed on one card (4 ranks share it through the
# tenancy lock; RCCL refuses duplicate devices, so the exchange falls back to gloo)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
LFM_BENCH_WATCHDOG=200 scripts/gpu_step.sh s2_share4 280 python -u bench.py --gpus 4 --share-gpus --steps 3 --warmup 1 || exit $?
echo done
