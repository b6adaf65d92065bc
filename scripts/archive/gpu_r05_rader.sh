# Round 5: Rader's algorithm for primes — parity tests, the prime3001 bench
# line (production dispatch vs the chirp-z plan), a prime sweep and the
# rocprofv3 kernel stats of the prime3001 workload.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "rader or plan_kinds or jit_specialisations or chirpz6k or primes or chirpz_plan" > gpurun_out/r05/pytest_rader.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_rader.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload prime3001 --steps 20 --warmup 3 > gpurun_out/r05/bench_prime3001.json 2> gpurun_out/r05/bench_prime3001.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/r05/bench_prime3001.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05/bench_prime3001.err; exit $rc; }
timeout -k 10 400 python -u scripts/bench_rader.py > gpurun_out/r05/rader_sweep.jsonl 2> gpurun_out/r05/rader_sweep.err; rc=$?
echo "sweep rc=$rc"; cat gpurun_out/r05/rader_sweep.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05/rader_sweep.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05/prof_prime3001 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload prime3001 --steps 20 --warmup 3 --cpu-seconds 0 --config-cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/r05/prof_prime3001.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
