# Round 5: the wave-resident Pwelch kernel (pwelch_wave.hip, F <= 1024)
# against the previous kernels (lib_pwoff), with and without the next group in
# flight (lib_nopf); parity first. Rader's chunked loads for short primes.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05/pytest_pww.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pww.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:1024 4096:2048"
for r in 1 2; do
for L in default lib_pwoff lib_nopf; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  echo "== $L round $r"
  timeout -k 10 300 python -u scripts/bench_pwelch.py $CASES > gpurun_out/r05/pww_$L.$r.jsonl 2>gpurun_out/r05/pww_$L.err; rc=$?
  cat gpurun_out/r05/pww_$L.$r.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05/pww_$L.err; exit $rc; }
done
done
unset GDSP_LIB
timeout -k 10 300 python -u scripts/bench_rader.py 17 19 23 37 101 257 641 > gpurun_out/r05/rader_small.jsonl 2> gpurun_out/r05/rader_small.err; rc=$?
echo "rader rc=$rc"; cat gpurun_out/r05/rader_small.jsonl
exit $rc
