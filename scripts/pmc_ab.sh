#!/bin/bash
# PMC HBM bytes (FETCH_SIZE, WRITE_SIZE; separate passes, counters only, schedule 3 event-
# ordered) of bench.py for each library named (built in-tree; LFM_LIBRARY selects it).
# Usage on the GPU box: bash scripts/pmc_ab.sh liblfm liblfm_x ...; then
# python scripts/pmc_ab_summary.py liblfm liblfm_x ... in the container.
set -u
export TMPDIR=/tmp
for lib in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LFM_LIBRARY=dis_project_amd/$lib.so LFM_S3_EVENTS=1 scripts/gpu_step.sh pmc_${lib}_$c 120 \
      rocprofv3 --pmc $c -d gpurun_out/pmc_${lib}_$c -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit $?
  done
done
