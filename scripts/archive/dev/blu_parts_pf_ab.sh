# output-split chirp-z row touch-ahead: measured with lib_pp<D> (-DGDSP_BLU_PF_PARTS=<D> rows ahead; now 2 by default, 0 = none)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_pp4/libgdspfft.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "output_parts" > gpurun_out/pp_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/pp_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in default go-dsp_amd/lib_pp2 go-dsp_amd/lib_pp4 go-dsp_amd/lib_pp8; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_sizes.py 8209 11003 12289 14563 > gpurun_out/sz.jsonl 2>&1 || exit $?
  echo "$L $(grep '"chirpz": false' gpurun_out/sz.jsonl | python -c "import sys,json;print(' '.join('%d:%.3f'%(d['n'],d['ms']) for d in map(json.loads,sys.stdin)))")"
done
done
