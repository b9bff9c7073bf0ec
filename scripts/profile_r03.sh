#!/bin/bash
# Round-3 profile set (GPU box, repo root): rocprofv3 kernel traces + PMC byte counters of
#   c2  the bench.py default (schedule 3, fused gram)       prof_trace / prof_fetch / prof_write
#   c4  the fp32 N = 65536 gram fill (bench.py --workload c4)  prof_c4 / prof_c4_write
#   c2 with LFM_GRAM_FUSE=0 (the fp64 gram as its own kernel) prof_unfused / prof_unfused_write
# then the untraced bench lines of c2 / c3 / c4 / c5, the MLL step timeline and unit trace,
# value_and_grad timing, the C3 concurrency rates (farm.choose_workers' table) and the
# vendor-library reference points.
# PMC passes run event-ordered (LFM_S3_EVENTS=1: device-side cross-stream waits cannot be met
# under the counters' serialised dispatch), one counter per pass.
set -u
export TMPDIR=/tmp
R=${1:-r03}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline"
scripts/gpu_step.sh prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace \
  -o run --output-format csv -- $B --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/prof_trace.log | tail -1 > gpurun_out/prof_trace_bench.json || exit $?
LFM_S3_EVENTS=1 scripts/gpu_step.sh prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch \
  -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
LFM_S3_EVENTS=1 scripts/gpu_step.sh prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write \
  -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
scripts/gpu_step.sh prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 \
  -o run --output-format csv -- $B --workload c4 --steps 5 --warmup 1 || exit $?
grep '^{' gpurun_out/prof_c4.log | tail -1 > gpurun_out/prof_c4_bench.json || exit $?
scripts/gpu_step.sh prof_c4_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_c4_write \
  -o run --output-format csv -- $B --workload c4 --steps 2 --warmup 1 --no-profile || exit $?
LFM_GRAM_FUSE=0 scripts/gpu_step.sh prof_unfused 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unfused \
  -o run --output-format csv -- $B --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/prof_unfused.log | tail -1 > gpurun_out/prof_unfused_bench.json || exit $?
LFM_GRAM_FUSE=0 LFM_S3_EVENTS=1 scripts/gpu_step.sh prof_unfused_write 300 rocprofv3 --pmc WRITE_SIZE \
  -d gpurun_out/prof_unfused_write -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
scripts/gpu_step.sh bench_c2 300 python bench.py --steps 20 --warmup 5 || exit $?
scripts/gpu_step.sh bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 1 || exit $?
scripts/gpu_step.sh bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 || exit $?
scripts/gpu_step.sh bench_c5 300 python bench.py --workload c5 --steps 20 --warmup 3 || exit $?
scripts/gpu_step.sh timeline 180 python scripts/step_timeline.py --json gpurun_out/${R}_step_timeline.json || exit $?
scripts/gpu_step.sh unit_trace 180 python -u scripts/unit_trace.py gpurun_out/${R}_unit_trace.npz || exit $?
scripts/gpu_step.sh grad_time 300 python scripts/grad_time.py || exit $?
for k in 1 2 3 4; do
  scripts/gpu_step.sh conc_s1_$k 300 python scripts/concurrency_probe.py $k 3 || exit $?
done
PROBE_SCHED=3 scripts/gpu_step.sh conc_s3_1 300 python scripts/concurrency_probe.py 1 3 || exit $?
scripts/gpu_step.sh library_ref 300 python -u scripts/library_ref.py --json gpurun_out/${R}_library_ref.json || exit $?
echo done
