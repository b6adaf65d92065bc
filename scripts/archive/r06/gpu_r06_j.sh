# Round 6: the chirp-z pass-B table as kept (RB 9, 10, 12-16, 18, 20, 21,
# 24, 25): its parity tests, then the non-smooth sweep's default list.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06j
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz or plan_kinds or rader or convolve or random_lengths" > gpurun_out/r06j/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06j/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 scripts/sweep_nonsmooth.py > gpurun_out/r06j/nonsmooth_sweep.jsonl 2> gpurun_out/r06j/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06j/sweep.err; exit $rc; }
