#!/bin/bash
# Round 3: vendor-library reference points and a per-workgroup trace of one C2 MLL
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/library_ref.py --json gpurun_out/library_ref.json > gpurun_out/library_ref.log 2>&1
timeout -k 10 180 python -u scripts/unit_trace.py gpurun_out/unit_trace_c2.npz > gpurun_out/unit_trace.log 2>&1
