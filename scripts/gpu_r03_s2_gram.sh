#!/bin/bash
# Round 3, session 2: gram fill variants (rows per workgroup, nontemporal stores), timed and
# checked bit-identical on sampled rows
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_step.sh s2_gram_ab 400 python -u scripts/gram_ab.py "LFM_GRAM_R=64" "LFM_GRAM_R=64 LFM_GRAM_NT=1" "LFM_GRAM_R=128" "LFM_GRAM_R=128 LFM_GRAM_NT=1" "LFM_GRAM_R=256" "LFM_GRAM_R=256 LFM_GRAM_NT=1" || exit $?
echo done
