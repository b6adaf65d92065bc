# Round-4 closing evidence in ONE gpurun session: the
# driver-style default bench line, then rocprofv3 --kernel-trace --stats of the
# five BASELINE workloads (20 timed + 3 warm-up launches, as bench.py), the HBM
# PMC passes (FETCH_SIZE, WRITE_SIZE) and the SQ counter passes of the same
# workloads. Summaries are turned into profiles/r04/ by tools/*_summary.py on
# the CPU side afterwards.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_default.err; exit $rc; }
bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch || exit 1
bash scripts/gpu_pmc_r03.sh radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch || exit 1
cd $GRAFT_REPO_ROOT && bash scripts/gpu_sq.sh radix4096 bluestein3000 chirpz3000 pwelch fft2_8192
