#!/bin/bash
# Round 3, session 2: full -m gpu suite after the ctypes pointer change, C5 / C2 bench lines
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_host_suite 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh s2_bench_c2 300 python bench.py --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh s2_rccl_c5 200 python -u bench.py --gpus 2 --share-gpus --workload c5 --steps 10 --warmup 2 || exit $?
echo done
