# Round 6 A/B, not kept: the small kernels' grid-table pass with each kind of
# entry whole within a wave (LFM_TABLE_WAVES, since removed) against the strided loop
# (ablibs/notw, built with -DLFM_TABLE_WAVES=0), plus the fit / MLL phase stamps of that build.
# The variant's source is gone; this script is the record of how it was measured.
export TMPDIR=/tmp
S=scripts/gpu_step.sh
LFM_LIBRARY=ablibs/fitst/liblfm.so $S r06g_fitst 200 python -u scripts/fit_stamps.py 150 c5 || exit $?
LFM_LIBRARY=ablibs/stamps/liblfm.so $S r06g_stamps 200 python -u scripts/small_stamps.py || exit $?
for r in 1 2; do
  for lib in ablibs/notw/liblfm.so dis_project_amd/liblfm.so; do
    tag=$(basename $(dirname $lib))
    LFM_LIBRARY=$lib $S r06g_c5_${tag}_$r 120 python -u bench.py --workload c5 --steps 2000 --warmup 200 --no-cpu-baseline || exit $?
    LFM_LIBRARY=$lib $S r06g_c5fit_${tag}_$r 120 python -u bench.py --workload c5fit --steps 30 --warmup 3 --no-cpu-baseline || exit $?
  done
done
$S r06g_tests 400 python -u -m pytest tests/test_farm.py tests/test_gpu_batch_grad.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
echo done
