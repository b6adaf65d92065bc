# Round 5, late: the last Pwelch-only lists as the batched FFT's lists too
# (lib_f2, tools/spec_variants.py) against the current FFT lists: batched FFT
# and Rader on the primes n + 1 that use them; two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_f2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py 500 625 375 250 200 320 1152 > $R/gpurun_out/r05/f2_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $R/gpurun_out/r05/f2_fft_$L.$r.jsonl | python3 -c "import sys,json; print(' '.join(f\"{d['n']}:{d['ms']:.3f}\" for d in map(json.loads,sys.stdin)))"
  timeout -k 10 300 python3 $R/scripts/bench_rader.py 251 1153 > $R/gpurun_out/r05/f2_rader_$L.$r.jsonl 2>&1; rc=$?
  echo "== rader $L $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $R/gpurun_out/r05/f2_rader_$L.$r.jsonl | python3 -c "import sys,json; print(' '.join(f\"{d['n']}:{d['ms']:.3f}k{d['kind']}\" for d in map(json.loads,sys.stdin)))"
done
done
