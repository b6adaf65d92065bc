# Round 5, end: the production size map (scripts/bench_sizes_default.py) and
# the Rader-vs-chirp-z sweep over primes at the final sources.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u scripts/bench_sizes_default.py > gpurun_out/r05/sizes_default.jsonl 2> gpurun_out/r05/sizes_default.err; rc=$?
echo "sizes rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05/sizes_default.err; exit $rc; }
timeout -k 10 600 python -u scripts/bench_rader.py > gpurun_out/r05/rader_sweep_final.jsonl 2> gpurun_out/r05/rader_sweep_final.err; rc=$?
echo "rader rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05/rader_sweep_final.err; exit $rc; }
