#!/bin/bash
# Round 6's GPU steps, one named study per argument (each step under its own time limit via
# scripts/gpu_step.sh; the first failing step ends the call — never retried):
#   tests    the whole -m gpu suite, then smoke()
#   handoff  the small kernels before / after the wave hand-off hardening (ablibs/r05 = round 5's
#            library, ablibs/nohandoff = this tree with -DLFM_WAVE_HANDOFF=0), c5 and c5fit bench
#            lines interleaved, two rounds
#   rehearse two ranks sharing the card, gloo exchange: c5 (16 rounds per rank) and c5fit
#            (the 15 fits partitioned)
#   overlap  the restart pipeline's tests and c3 lines off / on at several tail starts / reserves
#   ovltrace rocprofv3 kernel traces of the c3 step with the pipeline off / on
#   c2 c3 c5 c5fit   one bench line each (the default step counts of the round's profile set)
# The studies `mixed` (schedule-1 fillers, bench --mixed) and `overlap2`-`overlap4` (pipeline
# priority, prologue chains on the reserve, two prologue launches, a head of launch 1 on the
# overlap stream) ran at commits 4b52ebb / a3c0876 / 292617b / 5183b09; their knobs measured
# slower or equal and were removed (profiles/r06_ab.txt).
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
for study in "$@"; do
  case $study in
    tests)
      $S r06_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
      $S r06_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
      ;;
    handoff)
      for r in 1 2; do
        for lib in ablibs/r05/liblfm.so ablibs/nohandoff/liblfm.so dis_project_amd/liblfm.so; do
          tag=$(basename "$(dirname "$lib")")
          LFM_LIBRARY=$lib $S r06_handoff_c5_${tag}_$r 120 python -u bench.py --workload c5 --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
          LFM_LIBRARY=$lib $S r06_handoff_c5fit_${tag}_$r 120 python -u bench.py --workload c5fit --steps 30 --warmup 3 --no-cpu-baseline || exit $?
        done
      done
      ;;
    rehearse)
      R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
      $S r06_reh_c5 300 $R --master-port 29532 bench.py --gpus 2 --workload c5 --steps 500 --warmup 50 \
        --share-gpus --gather gloo --no-cpu-baseline || exit $?
      $S r06_reh_c5fit 300 $R --master-port 29533 bench.py --gpus 2 --workload c5fit --steps 5 --warmup 1 \
        --share-gpus --gather gloo --no-cpu-baseline || exit $?
      ;;
    overlap)
      # C3's restart pipeline (lfm_mll_multi_f64): its tests, then c3 lines with it off / on at
      # several tail starts and reserves, interleaved, two rounds
      $S r06_ovl_tests 400 python -u -m pytest tests/test_gpu_full.py -m gpu -x -v --timeout 200 --timeout-method thread -k pipeline || exit $?
      for r in 1 2; do
        for v in "LFM_OVERLAP=0" "LFM_OVERLAP=1" "LFM_OVL_AT=8192" "LFM_OVL_AT=4096" "LFM_OVL_RESERVE=32" "LFM_OVL_RESERVE=128"; do
          tag=${v//=/_}
          env $v $S r06_ovl_${tag}_$r 300 python -u bench.py --workload c3 --steps 4 --warmup 1 --no-cpu-baseline || exit $?
        done
      done
      ;;
    ovltrace)
      # kernel traces of the C3 step with the pipeline off / on (reserve 96): each kernel's
      # queue, start and end (scripts/ovl_timeline.py)
      for v in 0 1; do
        export LFM_OVERLAP=$v LFM_OVL_RESERVE=96
        $S r06_ovltrace_$v 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_ovltrace_$v -o run -- \
          python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit $?
      done
      unset LFM_OVERLAP LFM_OVL_RESERVE
      ;;
    fitab)
      for r in 1 2; do
        for lib in ablibs/r05/liblfm.so dis_project_amd/liblfm.so; do
          tag=$(basename "$(dirname "$lib")")
          LFM_LIBRARY=$lib $S r06_fitab_${tag}_$r 120 python -u bench.py --workload c5fit --steps 30 --warmup 3 --no-cpu-baseline || exit $?
        done
      done
      ;;
    c2) $S r06_bench_c2 300 python -u bench.py --workload c2 --steps 20 --warmup 3 || exit $? ;;
    c3) $S r06_bench_c3 400 python -u bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline || exit $? ;;
    c5) $S r06_bench_c5 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 || exit $? ;;
    c5fit) $S r06_bench_c5fit 300 python -u bench.py --workload c5fit --steps 30 --warmup 3 || exit $? ;;
    *) echo "unknown study $study"; exit 2 ;;
  esac
done
echo done
