# Round 6: the whole GPU suite and smoke on the final tree (as the driver runs them).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06x
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r06x/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06x/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06x/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/r06x/smoke.log; [ $rc -eq 0 ] || exit $rc
