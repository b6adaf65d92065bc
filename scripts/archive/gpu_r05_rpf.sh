# Round 5: the Rader kernel with an L2 touch-ahead of the row 16 blocks on
# (default) against none (lib_rpf0), prime3001 bench line, alternating; the
# Rader GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "rader or primes" > gpurun_out/r05/pytest_rpf.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05/pytest_rpf.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
for L in default lib_rpf0; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python bench.py --workload prime3001 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
  [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['parity']['max_nrel_vs_oracle'])" | tee -a gpurun_out/r05/rader_pf_ab.txt
done
done
for L in default lib_rpf0; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_rader.py 37 257 1009 2053 3001 4001 7681 8191 > gpurun_out/r05/rader_pf_sweep_$L.jsonl 2> gpurun_out/r05/rader_pf_sweep_$L.err; rc=$?
  echo "sweep $L rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r05/rader_pf_sweep_$L.err; exit $rc; }
done
