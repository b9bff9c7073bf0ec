#!/bin/bash
# Round profile set (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats of bench.py (5 timed + 2 warm C2 evaluations); the
#      traced run's own JSON line is kept beside the stats (gpurun_out/prof_trace_bench.json)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE), counters only, schedule 3 event-ordered
#   3. summarize_profile.py: profiles/syrk_traffic.json (read by bench.py's roofline.traffic)
#   4. the untraced bench.py (default workload, with the CPU baseline) -> gpurun_out/bench_<R>.json
#   5. per-step device-stamp timelines of the MLL and of value_and_grad's bordered factor
#      (per-launch TF/s), the chain's phase stamps, value_and_grad timing, the C3 / C5 lines
# Each GPU step has its own time limit; the script stops at the first failure. Afterwards run
# `python scripts/summarize_profile.py <R> gpurun_out/bench_<R>.json` in the container to
# regenerate the same profiles/ files from the merged gpurun_out/.
set -u
export TMPDIR=/tmp
R=${1:-r02}
STEPS=${STEPS:-10}
scripts/gpu_step.sh prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace \
  -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline || exit $?
grep '^{' gpurun_out/prof_trace.log | tail -1 > gpurun_out/prof_trace_bench.json || exit $?
LFM_S3_EVENTS=1 scripts/gpu_step.sh prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch \
  -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit $?
LFM_S3_EVENTS=1 scripts/gpu_step.sh prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write \
  -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit $?
python scripts/summarize_profile.py $R > gpurun_out/summary_pre.log 2>&1 || exit $?
scripts/gpu_step.sh bench 600 python bench.py --steps $STEPS --warmup 2 || exit $?
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench_$R.json || exit $?
scripts/gpu_step.sh timeline 120 python scripts/step_timeline.py --json gpurun_out/${R}_step_timeline.json || exit $?
scripts/gpu_step.sh timeline_grad 120 python scripts/step_timeline.py --grad --json gpurun_out/${R}_step_timeline_grad.json || exit $?
scripts/gpu_step.sh chain_stamps 120 python scripts/chain_stamps.py || exit $?
scripts/gpu_step.sh grad_time 120 python scripts/grad_time.py || exit $?
scripts/gpu_step.sh bench_c3 300 python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
scripts/gpu_step.sh bench_c5 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline || exit $?
echo done
