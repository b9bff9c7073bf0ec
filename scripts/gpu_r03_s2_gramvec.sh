#!/bin/bash
# Round 3, session 2: gram fill with 16-B stores (LFM_GRAM_VEC) — A/B with bit-identity, tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_gramvec_ab 400 python -u scripts/gram_ab.py "LFM_GRAM_VEC=0" "LFM_GRAM_VEC=1" || exit $?
scripts/gpu_step.sh s2_gramvec_tests 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py tests/test_gpu_full.py -x -q --timeout 240 --timeout-method thread || exit $?
scripts/gpu_step.sh s2_gramvec_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 || exit $?
echo done
