# Round 6: kind 8 and the smooth-L chirp-z under the plan-time race: their
# parity tests, the plan-kind / chirp-z / random-length tests, then the
# non-smooth sweep (production plan against the forced chirp-z plan).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06d
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "smooth_l" > gpurun_out/r06d/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r06d/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/sweep_nonsmooth.py > gpurun_out/r06d/nonsmooth_sweep.jsonl 2> gpurun_out/r06d/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r06d/sweep.err; exit $rc; }
timeout -k 10 300 python -u scripts/sweep_nonsmooth.py 4111 4253 4507 4621 4801 5003 5209 5519 5851 6007 6143 1559 1777 1999 3331 3583 3851 > gpurun_out/r06d/blufix_sweep.jsonl 2>> gpurun_out/r06d/sweep.err; rc=$?
echo "sweep2 rc=$rc"; exit $rc
