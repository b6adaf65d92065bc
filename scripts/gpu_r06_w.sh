# Round 6: the fused chirp-z parity test with its in-place check.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06w
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz6k_vs_oracle" > gpurun_out/r06w/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06w/pytest.log; [ $rc -eq 0 ] || exit $rc
