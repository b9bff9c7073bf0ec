scripts/gpu_step.sh tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
timeout -k 10 60 python scripts/probe_potrf.py > gpurun_out/potrf.log 2>&1 || exit 1
cat gpurun_out/potrf.log | tr '\n' ' '; echo
export LFM_SCHED=3
for v in "16 1 0" "16 1 1" "0 1 0" "16 1 0" "24 1 0"; do
 set -- $v
 LFM_SIDE_CUS=$1 LFM_TALL_POS=$2 LFM_STEP_EXP=$3 timeout -k 10 100 python scripts/chol_sweep.py 1,$1 > gpurun_out/tp.log 2>&1 || exit 1
 echo "$v $(cut -c150-230 gpurun_out/tp.log)"
done
