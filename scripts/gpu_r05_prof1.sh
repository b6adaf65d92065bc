# Round 5, first evidence session: the default bench line (every BASELINE
# config nested, prime3001 and pwelch_default new), rocprofv3 kernel stats of
# each workload, SQ counters of the new kernels, and an A/B of Rader radix
# lists for the prime 3001 (variant libraries lib_rad_*).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05/bench_default.err; exit $rc; }
for r in 1 2; do
for L in default lib_rad_b lib_rad_c lib_rad_d lib_rad_e lib_rad_f; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python bench.py --workload prime3001 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
  [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['parity']['max_nrel_vs_oracle'],d.get('chirpz',{}).get('ms_per_step'))" | tee -a gpurun_out/r05/rader_radix_ab.txt
done
done
unset GDSP_LIB
bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 prime3001 fft2_8192 pwelch pwelch_default || exit 1
cd $GRAFT_REPO_ROOT && bash scripts/gpu_sq.sh prime3001 pwelch_default
