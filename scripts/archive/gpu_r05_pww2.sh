# Round 5: the wave-resident Pwelch kernel after the branch-free loads and
# LDS twiddle bases, against the previous kernels (lib_pwoff) and without the
# next group in flight (lib_nopf); Pwelch parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pww2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pww2.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:1024"
for r in 1 2; do
for L in default lib_pwoff lib_nopf; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  echo "== $L round $r"
  timeout -k 10 300 python -u scripts/bench_pwelch.py $CASES > gpurun_out/r05/pww2_$L.$r.jsonl 2>gpurun_out/r05/pww2_$L.err; rc=$?
  cat gpurun_out/r05/pww2_$L.$r.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05/pww2_$L.err; exit $rc; }
done
done
