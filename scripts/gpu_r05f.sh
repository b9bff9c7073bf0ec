#!/bin/bash
# round 5: the last small-kernel commit's GPU tests, then the C4 fill study:
# store-shape / leading-dimension A/B (ablibs/gram, -DLFM_GRAM_AB) and PMC passes on the c4 fill
set -u
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=scripts/gpu_step.sh
B="python3 bench.py --no-cpu-baseline --workload c4"
$S r05f_tests 600 python -u -m pytest tests/test_gpu_batch_grad.py tests/test_farm.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
LFM_LIBRARY=ablibs/gram/liblfm.so $S r05f_gram_ab 300 python -u scripts/gram_ab.py "" LFM_GRAM_AB=1 \
  LFM_GRAM_AB=2 LFM_GRAM_AB=3 PAD=64 PAD=1024 "LFM_GRAM_AB=1 PAD=64" || exit $?
$S r05f_pmc_sq 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/r05f_pmc_sq -o run --output-format csv -- \
  $B --steps 2 --warmup 1 --no-profile || exit $?
$S r05f_pmc_tcc 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum SQ_INSTS_LDS SQ_INSTS_VALU \
  SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/r05f_pmc_tcc -o run --output-format csv -- \
  $B --steps 2 --warmup 1 --no-profile || exit $?
echo done
