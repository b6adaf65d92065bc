# Round 6: the kept four-pass entries ((6,6), (8,5), (8,6), (8,8)): parity of
# the chirp-z, Rader, random-length and size tests, then the sweep against the
# previous library on lengths across 4097 ... 8192, the gaps included.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06t
cd $R
timeout -k 10 800 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz_smooth or plan_kinds or rader or convolve or random_lengths or sizes" > gpurun_out/r06t/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06t/pytest.log; [ $rc -eq 0 ] || exit $rc
N="4099 4603 4621 5119 5147 5351 5381 5749 5779 6143 6151 6911 7159 7673 8059 8069 8191"
for r in 1 2; do
  for L in lib_base lib; do
    GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/sweep_nonsmooth.py $N > gpurun_out/r06t/${L}_$r.jsonl 2> gpurun_out/r06t/sweep.err; rc=$?
    echo "$L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06t/sweep.err; exit $rc; }
  done
done
