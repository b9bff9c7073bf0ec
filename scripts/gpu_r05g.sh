#!/bin/bash
# round 5: C4 fill, persistent-grid variant and isolated (bench-like) vs back-to-back timing,
# with rocprofv3 kernel traces of the two timing modes
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
export LFM_LIBRARY=ablibs/gram/liblfm.so
$S r05g_gram_ab 300 python -u scripts/gram_ab.py "" ISO=200 LFM_GRAM_AB=4 "LFM_GRAM_AB=4 LFM_GRAM_AB_WG=4096" \
  "LFM_GRAM_AB=4 LFM_GRAM_AB_WG=1024" "LFM_GRAM_AB=4 ISO=200" || exit $?
$S r05g_trace_b2b 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05g_trace_b2b -o run --output-format csv -- \
  python3 scripts/gram_ab.py "" || exit $?
$S r05g_trace_iso 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r05g_trace_iso -o run --output-format csv -- \
  python3 scripts/gram_ab.py ISO=200 || exit $?
echo done
