#!/bin/bash
# Round 3, session 2: the RCCL-failure fallback on one card (two ranks sharing device 0: RCCL
# refuses the duplicate GPU, both ranks fall back to gloo); stacks dumped if it hangs
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
LFM_BENCH_WATCHDOG=90 NCCL_DEBUG=WARN scripts/gpu_step.sh s2_rccl_share2 150 python -u bench.py --gpus 2 --share-gpus --steps 3 --warmup 1 || exit $?
echo done
