# Round-4: full GPU parity suite (default build + the development build's
# tests) and smoke(), as the driver runs them; logs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
(git log -1 --format=%H 2>/dev/null || echo "HEAD $(date)") > gpurun_out/pytest_gpu.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread >> gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
exit $rc
