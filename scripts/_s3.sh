scripts/gpu_step.sh tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
run() { timeout -k 10 100 python scripts/chol_sweep.py 1,32 > gpurun_out/tp.log 2>&1 || exit 1; python -c "import json,sys; d=json.loads(open('gpurun_out/tp.log').read().strip().splitlines()[-1]); print(sys.argv[1:], round(d['ms_median'],3), round(d['ms_min'],3), d['mll'])" "$@"; }
for v in ${S3_VARIANTS:-"LFM_CHAIN_SMALL=0" "LFM_CHAIN_SMALL=3"}; do export $v; run $v; done
timeout -k 10 100 python scripts/chain_stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
sed -n '1,3p;29,31p;48,51p' gpurun_out/stamps.log; tail -1 gpurun_out/stamps.log
