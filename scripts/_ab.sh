timeout -k 10 400 python scripts/ab.py "$@" > gpurun_out/ab.log 2>&1; rc=$?; tail -n 12 gpurun_out/ab.log; exit $rc
