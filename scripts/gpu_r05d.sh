#!/bin/bash
# round 5: the farm tests (device-side round), the c5 bench line with the chained 1-rank round
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_farm.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05d_farm.log 2>&1 || { tail -60 gpurun_out/r05d_farm.log; exit 1; }
tail -3 gpurun_out/r05d_farm.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 > gpurun_out/r05d_c5.json 2> gpurun_out/r05d_c5.err || { tail -20 gpurun_out/r05d_c5.err; exit 3; }
cat gpurun_out/r05d_c5.json
