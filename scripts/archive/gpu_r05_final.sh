# Round 5, final: the whole GPU suite, smoke and the driver-style default bench
# line at the closing sources.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05f
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05f/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05f/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r05f/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05f/bench_default.json 2> gpurun_out/r05f/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05f/bench_default.err; exit $rc; }
tail -c 300 gpurun_out/r05f/bench_default.json
