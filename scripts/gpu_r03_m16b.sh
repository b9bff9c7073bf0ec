#!/bin/bash
# Round 3: the full -m gpu suite and the bench lines on the 16x16x4 tile body
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu_m16 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh bench_c2_m16 300 python bench.py --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh grad_m16 300 python scripts/grad_time.py || exit $?
echo done
