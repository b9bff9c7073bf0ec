export TMPDIR=/tmp
PROBE_T=126 PROBE_KD=512 PROBE_CIO=29 timeout -k 10 100 python scripts/probe_syrk.py > gpurun_out/gap_probe.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gap_trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/gap_bench.log 2>&1 || exit 1
PROBE_T=126 PROBE_KD=512 PROBE_CIO=29 timeout -k 10 100 python scripts/probe_syrk.py >> gpurun_out/gap_probe.log 2>&1 || exit 1
cat gpurun_out/gap_probe.log
