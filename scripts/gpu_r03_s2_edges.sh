#!/bin/bash
# round 3 session 2: edge-input parity tests + the tenancy tests after the lock-file change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_edges.py > gpurun_out/s2_edges.log 2>&1
rc=$?
tail -5 gpurun_out/s2_edges.log
exit $rc
