# CPU side after scripts/gpu_r04_close.sh: copy the closing session's
# rocprofv3 kernel stats, PMC and SQ summaries from gpurun_out/ into profiles/r04/.
set -e
cd "$(dirname "$0")/.."
mkdir -p profiles/r04
cp gpurun_out/bench_default.json profiles/r04/bench_default.json
for W in radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch; do
  cp gpurun_out/prof_$W/run_kernel_stats.csv profiles/r04/${W}_kernel_stats.csv
done
python3 tools/pmc_summary.py r04 radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch
python3 tools/trace_summary.py r04 20 radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch
python3 tools/sq_summary.py r04 radix4096 bluestein3000 chirpz3000 pwelch fft2_8192
