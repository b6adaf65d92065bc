# Round 5: after the 735 / 900 Pwelch-only lists: the Pwelch and
# specialisation GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pwelch or Pwelch or mixed or specialisation" > gpurun_out/r05/pytest_verify6.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify6.log; [ $rc -eq 0 ] || exit $rc
