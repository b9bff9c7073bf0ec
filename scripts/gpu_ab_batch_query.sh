set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; S=scripts/gpu_step.sh
$S q_tests 300 python -u -m pytest tests/test_farm.py tests/test_gpu_batch_grad.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
for i in 1 2 3; do
  $S q_new_$i 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
  LFM_LIBRARY=ablibs/prevq/liblfm.so $S q_old_$i 300 python -u bench.py --workload c5 --steps 3000 --warmup 300 --no-cpu-baseline || exit $?
done
echo done
