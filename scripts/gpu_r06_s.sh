# Round 6: the four-pass fused chirp-z (chirpz4_kernel, M = 16 R1 R2 16 for
# 3201 <= n <= 8192): parity, then the sweep on the product library and the
# previous one (go-dsp_amd/lib_base), alternating, on the first and last
# prime of each (R1, R2) range.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06s4
cd $R
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz6k or chirpz_plan" > gpurun_out/r06s4/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06s4/pytest.log; [ $rc -eq 0 ] || exit $rc
N="3203 3449 3457 3583 3593 3833 3847 4093 4099 4603 4621 5119 5147 5351 5381 5749 5779 6143 6151 6911 6917 7159 7177 7673 7681 8059 8069 8191"
for r in 1 2; do
  for L in lib_base lib; do
    GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/sweep_nonsmooth.py $N > gpurun_out/r06s4/${L}_$r.jsonl 2> gpurun_out/r06s4/sweep.err; rc=$?
    echo "$L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06s4/sweep.err; exit $rc; }
  done
done
