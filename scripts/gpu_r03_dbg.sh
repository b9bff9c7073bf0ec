#!/bin/bash
# Focused: the early-unit tests with a short device-wait bound (a stall reports its first wait
# kind in LFM_E_TIMEOUT's message within seconds), every case run (no -x).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
LFM_DEBUG_SPIN_LIMIT=4000000 scripts/gpu_step.sh early_dbg 500 python -u -m pytest tests/test_gpu_full.py -m gpu -v -k early --timeout 120 --timeout-method thread
grep -E "PASSED|FAILED|timed out" gpurun_out/early_dbg.log | head -60
