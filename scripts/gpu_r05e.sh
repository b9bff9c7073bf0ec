#!/bin/bash
# round 5: batched gradient / fit (two-wave problems), the small-kernel farm tests, c5 / c5fit lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_grad.py tests/test_farm.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05e_tests.log 2>&1 || { tail -60 gpurun_out/r05e_tests.log; exit 1; }
tail -3 gpurun_out/r05e_tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 > gpurun_out/r05e_c5.json 2> gpurun_out/r05e_c5.err || { tail -20 gpurun_out/r05e_c5.err; exit 3; }
timeout -k 10 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 > gpurun_out/r05e_c5fit.json 2> gpurun_out/r05e_c5fit.err || { tail -20 gpurun_out/r05e_c5fit.err; exit 4; }
cat gpurun_out/r05e_c5.json gpurun_out/r05e_c5fit.json
