run() { timeout -k 10 100 python scripts/chol_sweep.py "$@" > gpurun_out/tp.log 2>&1 || exit 1; python -c "import json,sys; d=json.loads(open('gpurun_out/tp.log').read().strip().splitlines()[-1]); print(sys.argv[1:], round(d['ms_median'],3), round(d['ms_min'],3), d['mll'])" "$@"; }
run 1,32
run 1,32,6144,1073741824,8192
run 1,32,6144,1073741824,10240
run 1,32,6144,1073741824,12288
run 1,32
