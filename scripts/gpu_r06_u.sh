# Round 6: the final chirp-z tables (three-pass RB 3-6, 9-16, 18-21, 24, 25;
# four-pass (6,6), (8,5), (8,6)): every chirp-z, Rader, random-length, size
# and Pwelch option test.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06u
cd $R
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz or plan_kinds or rader or convolve or random or sizes or pwelch" > gpurun_out/r06u/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06u/pytest.log; [ $rc -eq 0 ] || exit $rc
