timeout -k 10 100 python scripts/chain_stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
sed -n '1,3p;29,31p;45,51p' gpurun_out/stamps.log; tail -1 gpurun_out/stamps.log
