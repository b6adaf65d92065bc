# Round 6: real / imaginary LDS exchanges for one-row workgroups of the
# mixed-radix and Rader kernels (go-dsp_amd/lib_exp) against the product
# library: parity on the experiment library, then alternating bench lines
# and the sweep on Rader primes.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06k
cd $R
GDSP_LIB=$R/go-dsp_amd/lib_exp/libgdspfft.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rader or mixed or specs or sizes or c3k or jit" > gpurun_out/r06k/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06k/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh "bluestein3000 prime3001" "default go-dsp_amd/lib_exp" 3 || exit 1
for L in lib lib_exp; do
  GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/sweep_nonsmooth.py --no-chirpz 1153 1201 1409 2053 2689 3001 3329 1801 > gpurun_out/r06k/$L.jsonl 2> gpurun_out/r06k/sweep.err; rc=$?
  echo "sweep $L rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06k/sweep.err; exit $rc; }
done
