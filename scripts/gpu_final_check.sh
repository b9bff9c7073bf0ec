set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LFM_LIBRARY=ablibs/stamps/liblfm.so timeout -k 10 120 python -u scripts/small_stamps.py > gpurun_out/clk_stamps.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
echo done
