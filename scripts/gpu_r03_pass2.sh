#!/bin/bash
# Round 3, second GPU pass: the -m gpu suite, interleaved A/B of the early units, the four bench
# workloads with their CPU baselines, and the 2-rank self-launch rehearsal on one card.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh ab_early 400 env AB_ROUNDS=6 python scripts/ab.py "LFM_EARLY=0" "LFM_EARLY=30" "LFM_EARLY=18" "LFM_EARLY=42" "LFM_EARLY=30 LFM_EARLY_WMIN=1" "LFM_EARLY=12 LFM_EARLY_WMIN=1" || exit $?
scripts/gpu_step.sh bench_c2 300 python bench.py --steps 20 --warmup 5 || exit $?
scripts/gpu_step.sh bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 1 || exit $?
scripts/gpu_step.sh bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 || exit $?
scripts/gpu_step.sh bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh rehearse2 300 python bench.py --gpus 2 --share-gpus --gather gloo --steps 3 --warmup 1 || exit $?
echo done
