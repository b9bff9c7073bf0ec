scripts/gpu_step.sh tests 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
timeout -k 10 100 python scripts/chain_stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
sed -n '1,3p;46,50p' gpurun_out/stamps.log; tail -1 gpurun_out/stamps.log
bash scripts/_ab.sh "$@"
