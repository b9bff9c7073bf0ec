#!/bin/bash
# Round 3, session 2: rebuilt tree -> full -m gpu suite, smoke, C2 bench line
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/steps.log
scripts/gpu_step.sh s2_pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
scripts/gpu_step.sh s2_bench_c2 300 python bench.py --steps 20 --warmup 3 || exit $?
AB_ROUNDS=6 scripts/gpu_step.sh s2_ab_w2min 400 python -u scripts/ab.py "LFM_W2_MIN=5120" "LFM_W2_MIN=4096" "LFM_W2_MIN=3072" "LFM_W2_MIN=2048" "LFM_W2_MIN=1024" || exit $?
scripts/gpu_step.sh s2_rccl_share 300 python bench.py --gpus 2 --share-gpus --steps 3 --warmup 1 || exit $?
echo done
