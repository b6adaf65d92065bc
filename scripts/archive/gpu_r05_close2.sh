# Round-5 final closing evidence (as gpu_r05_close.sh, after the last kernel changes): the whole GPU suite, smoke, the
# driver-style default bench line, then rocprofv3 --kernel-trace --stats of
# every bench workload (20 timed + 3 warm-up launches, as bench.py) and the
# SQ counter passes of the kernels this round changed. Summaries become
# profiles/r05/ on the CPU side (tools/trace_summary.py, sq_summary.py).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05d
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05d/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05d/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r05d/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05d/bench_default.json 2> gpurun_out/r05d/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05d/bench_default.err; exit $rc; }
bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 prime3001 fft2_8192 pwelch pwelch_default || exit 1
cd $GRAFT_REPO_ROOT && bash scripts/gpu_sq.sh pwelch_default pwelch prime3001
