#!/bin/bash
# round 5, first GPU pass: the whole -m gpu suite, then the C2 and C5 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05a_suite.log 2>&1 || { tail -30 gpurun_out/r05a_suite.log; exit 1; }
tail -3 gpurun_out/r05a_suite.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r05a_c2.json 2> gpurun_out/r05a_c2.err || exit 2
timeout -k 10 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 > gpurun_out/r05a_c5.json 2> gpurun_out/r05a_c5.err || exit 3
cat gpurun_out/r05a_c2.json gpurun_out/r05a_c5.json
