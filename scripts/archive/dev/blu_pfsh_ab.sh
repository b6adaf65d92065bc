# chirp-z touch-ahead granularity: default (one load per 128 B) against
# lib_sh6 (per 64 B, -DGDSP_BLU_PF_SHIFT=6) and lib_pf0 (off, -DGDSP_BLU_PF=0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_sh6/libgdspfft.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "chirpz or prime" > gpurun_out/sh6_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/sh6_pytest.log)"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh chirpz3000 "default go-dsp_amd/lib_sh6 go-dsp_amd/lib_pf0" 3 || exit $?
for L in default go-dsp_amd/lib_sh6 go-dsp_amd/lib_pf0; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_sizes.py 61 251 1021 2039 4093 8191 > gpurun_out/sz.jsonl 2>&1 || exit $?
  echo "$L $(grep '"chirpz": true' gpurun_out/sz.jsonl | python -c "import sys,json;print(' '.join('%d:%.3f'%(d['n'],d['ms']) for d in map(json.loads,sys.stdin)))")"
done
