# Round 5, end: GPU tests touched by the last changes (Rader's thread limit,
# prime dimensions in Convolve / FFT2 / FFTN, the mixed-radix lists) and the
# whole parity file once more.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_verify.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify.log; [ $rc -eq 0 ] || exit $rc
