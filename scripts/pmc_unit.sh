set -u
export TMPDIR=/tmp PMC_T=127 PMC_KD=640 PMC_CIO=88
mkdir -p gpurun_out
python scripts/pmc_syrk.py 3 > gpurun_out/pmc_plain.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_u1 -o run --output-format csv -- python3 scripts/pmc_syrk.py 3 > gpurun_out/pmc_u1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_F64 -d gpurun_out/pmc_u2 -o run --output-format csv -- python3 scripts/pmc_syrk.py 3 > gpurun_out/pmc_u2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_u3 -o run --output-format csv -- python3 scripts/pmc_syrk.py 3 > gpurun_out/pmc_u3.log 2>&1 || exit $?
echo ok
