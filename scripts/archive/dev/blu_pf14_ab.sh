# chirp-z touch-ahead distance at M = 16384 (one block per CU): measured 16 (then default)
# against lib_p14d4 / lib_p14d8 (-DGDSP_BLU_PF14=<D>)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2; do
for L in default go-dsp_amd/lib_p14d4 go-dsp_amd/lib_p14d8; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_sizes.py 4099 5003 6007 8191 > gpurun_out/sz.jsonl 2>&1 || exit $?
  echo "$L $(python -c "import json;print(' '.join('%d:%.3f'%(d['n'],d['ms']) for d in map(json.loads,(l for l in open('gpurun_out/sz.jsonl') if l.startswith('{'))) if d['chirpz']))")"
done
done
