# Round 6: the kept chirp-z table (RB 3-6, 9, 10, 12-16, 18, 20, 21, 24, 25):
# parity of the chirp-z, Rader and random-length tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06o
cd $R
timeout -k 10 800 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz or plan_kinds or rader or convolve or random_lengths or sizes" > gpurun_out/r06o/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06o/pytest.log; [ $rc -eq 0 ] || exit $rc
