# Round 6: plan kind 8 (prime-factor Rader) parity, then the non-smooth sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06b
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "rader_pfa or plan_kinds" > gpurun_out/r06b/pytest_pfa.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r06b/pytest_pfa.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/sweep_nonsmooth.py > gpurun_out/r06b/nonsmooth_sweep.jsonl 2> gpurun_out/r06b/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r06b/sweep.err; exit $rc; }
