# Round 6: the fused chirp-z on every pass-B radix (chirpz6k.hpp, M = 256 RB
# for 1025 <= n <= 4096): its parity tests, then the non-smooth sweep on the
# new library and on the previous one (go-dsp_amd/lib_base, M = 6144 / 3072 /
# powers of 2), alternating, on the first and last prime of every RB range.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06h
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz6k or chirpz_plan or chirpz_smooth or plan_kinds or rader or convolve" > gpurun_out/r06h/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06h/pytest.log; [ $rc -eq 0 ] || exit $rc
N="1031 1151 1153 1279 1283 1399 1409 1531 1543 1663 1667 1789 1801 1913 1931 2039 2053 2297 2309 2557 2579 2687 2689 2803 2819 3067 3079 3191 3203 3323 3329 3583 3593 3833 3847 4093"
for r in 1 2; do
  GDSP_LIB=$R/go-dsp_amd/lib_base/libgdspfft.so timeout -k 10 400 python3 scripts/sweep_nonsmooth.py $N > gpurun_out/r06h/base_$r.jsonl 2> gpurun_out/r06h/sweep.err; rc=$?
  echo "base $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06h/sweep.err; exit $rc; }
  timeout -k 10 400 python3 scripts/sweep_nonsmooth.py $N > gpurun_out/r06h/new_$r.jsonl 2> gpurun_out/r06h/sweep.err; rc=$?
  echo "new $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06h/sweep.err; exit $rc; }
done
