#!/bin/bash
# Calibrates FETCH_SIZE / WRITE_SIZE for the trailing update's C tile access (8 B per lane,
# four 128-B row segments per instruction, nontemporal) on a known byte count: the step
# kernel's rest role over a full T = 127 triangle at depth 512 (lfm_probe_syrk bit 6), with C
# loaded (cio 88) and not loaded (cio 120); both store every lower C element once.
# Known bytes per launch: C = T (T + 1) / 2 * 128 * 128 * 8 read (88 only) and written (both).
# Usage on the GPU box: bash scripts/pmc_calib.sh; then python scripts/pmc_calib_summary.py.
set -u
export TMPDIR=/tmp
for cio in 88 120; do
  for c in FETCH_SIZE WRITE_SIZE; do
    PROBE_T=127 PROBE_KD=512 PROBE_CIO=$cio scripts/gpu_step.sh calib_${cio}_$c 120 \
      rocprofv3 --pmc $c -d gpurun_out/calib_${cio}_$c -o run --output-format csv -- \
      python3 scripts/probe_syrk.py || exit $?
  done
done
