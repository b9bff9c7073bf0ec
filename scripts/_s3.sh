scripts/gpu_step.sh tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
PROBE_T=126 PROBE_KD=512 PROBE_CIO=5,13 timeout -k 10 60 python scripts/probe_syrk.py || exit 1
run() { timeout -k 10 100 python scripts/chol_sweep.py "$@" > gpurun_out/tp.log 2>&1 || exit 1; python -c "import json,sys; d=json.loads(open('gpurun_out/tp.log').read().strip().splitlines()[-1]); print(sys.argv[1:], round(d['ms_median'],3), round(d['ms_min'],3), d['mll'])" "$@"; }
run 1,16
LFM_SCHED=1 run 1,0
scripts/gpu_step.sh bench 300 python bench.py --steps 10 --warmup 2 || exit $?
