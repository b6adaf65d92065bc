# Selected GPU tests: pytest -k "$1" (files $2, default tests), verbose, per-test timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_k.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_k.log | tail -40
exit $rc
