#!/bin/bash
# round 5: the new batched gradient / fit tests first, then the whole -m gpu suite, then benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_grad.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05b_batch.log 2>&1 || { tail -60 gpurun_out/r05b_batch.log; exit 1; }
tail -3 gpurun_out/r05b_batch.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05b_suite.log 2>&1 || { tail -40 gpurun_out/r05b_suite.log; exit 1; }
tail -3 gpurun_out/r05b_suite.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05b_c2.json 2> gpurun_out/r05b_c2.err || exit 2
timeout -k 10 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 > gpurun_out/r05b_c5.json 2> gpurun_out/r05b_c5.err || exit 3
cat gpurun_out/r05b_c2.json gpurun_out/r05b_c5.json
