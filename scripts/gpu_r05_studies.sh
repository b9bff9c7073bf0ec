#!/bin/bash
# Round 5's GPU studies behind profiles/r05_* (GPU box, repo root), one step per name:
#   bash scripts/gpu_r05_studies.sh STUDY...
# gram       C4 fill: store-shape / grid / leading-dimension A/B (ablibs/gram, make
#            EXTRA=-DLFM_GRAM_AB), its store-only floor and the runtime memset of the same bytes,
#            kernel traces back to back and bench-shaped (r05_ab_gram_*.txt, r05_gram.md)
# gram_pmc   C4 fill PMC passes: SQ wave-time split, stores, LDS, fabric write requests
#            (r05_gram_c4_pmc.txt)
# farm       the device-side farm round replayed from its graph and enqueued (LFM_FARM_GRAPH=0):
#            the farm tests, both c5 lines, a c5 kernel trace (r05_bench_c5_graph / _nograph.json)
# small      the small-kernel phase stamps: fit (ablibs/fitst, -DLFM_FIT_STAMPS=1) and MLL
#            (ablibs/stamps, -DLFM_SMALL_STAMPS=1) (r05_fit_phase_stamps.txt,
#            r05_c5_phase_stamps.txt), the fit / host-loop diagnostic, the pooled / C1 fit times
# pipe       the small factor's pipelined LDL^T columns against ablibs/nopipe (stamps, C5 lines,
#            the host split of a C5 step) (r05_ab_small_ldl.txt)
# tests      the batch-gradient tests twice, then the farm / parity / edge / regime tests
# Every step runs under its own time limit (scripts/gpu_step.sh); the first failure ends the run.
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
T="-m gpu -x -q --timeout 300 --timeout-method thread"
for study in "$@"; do
  case "$study" in
    gram)
      LFM_LIBRARY=ablibs/gram/liblfm.so $S gram_ab 300 python -u scripts/gram_ab.py "" \
        LFM_GRAM_AB=1 LFM_GRAM_AB=2 LFM_GRAM_AB=3 LFM_GRAM_AB=4 "LFM_GRAM_AB=4 LFM_GRAM_AB_WG=4096" \
        "LFM_GRAM_AB=4 LFM_GRAM_AB_WG=1024" LFM_GRAM_AB=5 MEMSET=1 ISO=200 PAD=64 PAD=1024 || exit $?
      LFM_LIBRARY=ablibs/gram/liblfm.so $S gram_trace_b2b 120 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/gram_trace_b2b -o run --output-format csv -- python3 scripts/gram_ab.py "" || exit $?
      LFM_LIBRARY=ablibs/gram/liblfm.so $S gram_trace_iso 120 rocprofv3 --kernel-trace --stats \
        -d gpurun_out/gram_trace_iso -o run --output-format csv -- python3 scripts/gram_ab.py ISO=200 || exit $?
      ;;
    gram_pmc)
      B="python3 bench.py --no-cpu-baseline --workload c4"
      $S gram_pmc_sq 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/gram_pmc_sq -o run \
        --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
      $S gram_pmc_tcc 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum SQ_INSTS_LDS \
        SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/gram_pmc_tcc -o run \
        --output-format csv -- $B --steps 2 --warmup 1 --no-profile || exit $?
      ;;
    farm)
      $S farm_tests 300 python -u -m pytest tests/test_farm.py $T || exit $?
      $S farm_c5 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
      LFM_FARM_GRAPH=0 $S farm_c5_nograph 300 python -u bench.py --workload c5 --steps 2000 --warmup 200 \
        --no-cpu-baseline || exit $?
      $S farm_c5_trace 180 rocprofv3 --kernel-trace --stats -d gpurun_out/farm_c5_trace -o run \
        --output-format csv -- python3 bench.py --workload c5 --steps 300 --warmup 30 --no-cpu-baseline || exit $?
      ;;
    small)
      LFM_LIBRARY=ablibs/fitst/liblfm.so $S fit_stamps 120 python -u scripts/fit_stamps.py 150 || exit $?
      LFM_LIBRARY=ablibs/fitst/liblfm.so $S fit_stamps_pooled 120 python -u scripts/fit_stamps.py 150 pooled || exit $?
      LFM_LIBRARY=ablibs/stamps/liblfm.so $S small_stamps 120 python -u scripts/small_stamps.py || exit $?
      $S fit_diag 200 python -u scripts/diag_fit.py || exit $?
      $S fit_pooled 200 python -u scripts/fit_pooled_time.py || exit $?
      $S c5fit 300 python -u bench.py --workload c5fit --steps 20 --warmup 3 || exit $?
      ;;
    pipe)
      # the one-wave factor's pipelined LDL^T columns (LFM_SMALL_PIPE, default) against ablibs/nopipe
      # (make EXTRA=-DLFM_SMALL_PIPE=0): the MLL kernel's phase stamps, C5 lines interleaved
      LFM_LIBRARY=ablibs/stamps/liblfm.so $S pipe_stamps 120 python -u scripts/small_stamps.py || exit $?
      for i in 1 2; do
        $S pipe_c5_on_$i 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
        LFM_LIBRARY=ablibs/nopipe/liblfm.so $S pipe_c5_off_$i 300 python -u bench.py --workload c5 \
          --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
      done
      $S pipe_split 200 python -u scripts/c5_host_split.py 3000 || exit $?
      ;;
    tests)
      $S tests_grad_a 300 python -u -m pytest tests/test_gpu_batch_grad.py $T || exit $?
      $S tests_grad_b 300 python -u -m pytest tests/test_gpu_batch_grad.py $T || exit $?
      $S tests_small 600 python -u -m pytest tests/test_farm.py tests/test_gpu_parity.py \
        tests/test_gpu_edges.py tests/test_gpu_regimes.py $T || exit $?
      ;;
    *) echo "unknown study $study"; exit 2 ;;
  esac
done
echo done
