# Round 6: the whole GPU suite, smoke and the default bench line at the
# current sources (the sources' stamp first, for the profiles' summaries).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06s
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
python3 tools/source_stamp.py > gpurun_out/source_stamp.json
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r06s/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06s/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06s/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r06s/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06s/bench_default.json 2> gpurun_out/r06s/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r06s/bench_default.err; exit $rc; }
tail -c 400 gpurun_out/r06s/bench_default.json
