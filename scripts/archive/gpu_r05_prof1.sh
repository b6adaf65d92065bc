# Round 5, first evidence session: the default bench line (every BASELINE
# config nested, prime3001 and pwelch_default new), rocprofv3 kernel stats of
# each workload and SQ counters of the new kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05/bench_default.err; exit $rc; }
# (the Rader radix-list A/B that ran here used temporary variant libraries;
# its result is profiles/r05/rader_radix_ab.txt)
bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 prime3001 fft2_8192 pwelch pwelch_default || exit 1
cd $GRAFT_REPO_ROOT && bash scripts/gpu_sq.sh prime3001 pwelch_default
