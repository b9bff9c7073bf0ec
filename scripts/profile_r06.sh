#!/bin/bash
# The profile set behind profiles/<R>_* (GPU box, repo root; R defaults to r06). Round 6 adds the
# GPU suite first, the C3 restart pipeline in the c3 line, the two-rank rehearsal and the c5 /
# c5fit lines with their threaded CPU baselines; round 5 added
# the c5fit line and the kernel traces of the c5 / c5fit workloads (the batch kernel, the
# device-side farm round's graph, the fit kernel). Every step runs
# on the current library under its own time limit (scripts/gpu_step.sh) and the script stops at
# the first failure. Then, on the container: scripts/summarize_profile.py R gpurun_out/prof_trace_bench.json
# and scripts/summarize_gram.py R turn the CSVs into profiles/R_*.
#   kernel traces (rocprofv3 --kernel-trace --stats) of
#     c2  bench.py's default (schedule 3, fused gram)          prof_trace
#     c4  the fp32 N = 65536 gram fill                          prof_c4
#     c2 with LFM_GRAM_FUSE=0 (the fp64 gram as its own kernel) prof_unfused
#     c5  the resident small-problem batch                      prof_c5
#   PMC passes, one counter group per pass, on the timed schedule's own launches serialised by
#   stream events (LFM_S3_EVENTS=2: every device-side cross-stream wait is met at dispatch, which
#   the counters' serialised dispatch needs): FETCH_SIZE and
#   WRITE_SIZE of c2, WRITE_SIZE of c4 and of the unfused gram, MFMA busy of the production unit
#   alone and of every c2 step launch
#   the bench lines of c2 / c3 / c4 / c5, the step timeline, the unit trace, value_and_grad
#   timing, the farm exchange latency (1-rank RCCL), the vendor-library reference points
set -u
export TMPDIR=/tmp
R=${1:-r06}
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline"
S=scripts/gpu_step.sh
$S ${R}_suite 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit $?
$S ${R}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace \
  -o run --output-format csv -- $B --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/prof_trace.log | tail -1 > gpurun_out/prof_trace_bench.json || exit $?
LFM_S3_EVENTS=2 $S prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch \
  -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
LFM_S3_EVENTS=2 $S prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write \
  -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
$S prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 \
  -o run --output-format csv -- $B --workload c4 --steps 5 --warmup 1 || exit $?
grep '^{' gpurun_out/prof_c4.log | tail -1 > gpurun_out/prof_c4_bench.json || exit $?
$S prof_c4_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_c4_write \
  -o run --output-format csv -- $B --workload c4 --steps 2 --warmup 1 --no-profile || exit $?
LFM_GRAM_FUSE=0 $S prof_unfused 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unfused \
  -o run --output-format csv -- $B --steps 5 --warmup 2 || exit $?
grep '^{' gpurun_out/prof_unfused.log | tail -1 > gpurun_out/prof_unfused_bench.json || exit $?
LFM_GRAM_FUSE=0 LFM_S3_EVENTS=2 $S prof_unfused_write 300 rocprofv3 --pmc WRITE_SIZE \
  -d gpurun_out/prof_unfused_write -o run --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
$S prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 \
  -o run --output-format csv -- $B --workload c5 --steps 200 --warmup 20 || exit $?
PMC_T=127 PMC_KD=640 PMC_CIO=88 $S mfma_unit 120 rocprofv3 --kernel-trace \
  --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/mfma_unit \
  -o run --output-format csv -- python3 scripts/pmc_syrk.py 3 || exit $?
LFM_S3_EVENTS=2 $S mfma_bench 180 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES \
  GRBM_GUI_ACTIVE -d gpurun_out/mfma_bench -o run --output-format csv -- \
  $B --steps 2 --warmup 1 --no-profile || exit $?
$S bench_c2 300 python bench.py --steps 20 --warmup 5 || exit $?
$S bench_c3 300 python bench.py --workload c3 --steps 5 --warmup 1 || exit $?
$S bench_c4 300 python bench.py --workload c4 --steps 10 --warmup 2 || exit $?
$S bench_c5 300 python bench.py --workload c5 --steps 2000 --warmup 200 || exit $?
$S bench_c5fit 300 python bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
$S prof_c5fit 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5fit \
  -o run --output-format csv -- $B --workload c5fit --steps 10 --warmup 2 || exit $?
$S timeline 180 python scripts/step_timeline.py --json gpurun_out/${R}_step_timeline.json || exit $?
$S unit_trace 180 python -u scripts/unit_trace.py gpurun_out/${R}_unit_trace.npz || exit $?
$S grad_time 300 python scripts/grad_time.py || exit $?
$S farm_latency 200 python scripts/farm_latency.py --json gpurun_out/${R}_allgather_latency.json \
  --rounds 3 dis_project_amd/liblfm.so || exit $?
$S library_ref 300 python -u scripts/library_ref.py --json gpurun_out/${R}_library_ref.json || exit $?
bash scripts/gpu_r06.sh rehearse || exit $?
echo done
