export LFM_SCHED=3
scripts/gpu_step.sh tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread || exit $?
for v in "16 1 0" "16 1 1" "0 1 0" "16 1 0" "24 1 0" "12 1 0"; do
 set -- $v
 LFM_SIDE_CUS=$1 LFM_TALL_POS=$2 LFM_STEP_EXP=$3 timeout -k 10 100 python scripts/chol_sweep.py 1,$1 > gpurun_out/tp.log 2>&1 || exit 1
 echo "$v $(cut -c150-230 gpurun_out/tp.log)"
done
