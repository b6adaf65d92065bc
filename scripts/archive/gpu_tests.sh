# Full GPU parity suite + smoke (what the driver runs at round end), no bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -1 gpurun_out/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -15
exit $rc
