#!/bin/bash
# Round 3: full -m gpu suite, bench lines and step timeline on the current kernels
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu_full2 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh bench_c2_full2 300 python bench.py --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh timeline_full2 200 python scripts/step_timeline.py --json gpurun_out/r03_step_timeline_v2.json || exit $?
scripts/gpu_step.sh trace_full2 200 python -u scripts/unit_trace.py gpurun_out/unit_trace_v2.npz || exit $?
scripts/gpu_step.sh grad_full2 300 python scripts/grad_time.py || exit $?
echo done
