# (measured with builds lib_pfall = touch in every block, lib_pfall8 = 4 blocks ahead;
# now the default: compare against scripts/build_variant.sh pf0 "-DGDSP_BLU_PF=0")
# chirp-z row touch-ahead for multi-transform blocks (M <= 4096): parity on the
# variant, then per-size timings (forced chirp-z, 2^27 samples) alternating builds
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_pf0/libgdspfft.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "chirpz or prime or random_lengths" > gpurun_out/pfall_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/pfall_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in default go-dsp_amd/lib_pf0; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_sizes.py 13 61 101 251 509 1021 2039 > gpurun_out/sz.jsonl 2>&1 || exit $?
  echo "$L $(grep '"chirpz": true' gpurun_out/sz.jsonl | python -c "import sys,json;print(' '.join('%d:%.3f'%(d['n'],d['ms']) for d in map(json.loads,sys.stdin)))")"
done
done
