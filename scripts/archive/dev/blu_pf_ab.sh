# chirp-z row prefetch A/B: build the no-prefetch variant first with
# scripts/build_variant.sh pf0 "-DGDSP_BLU_PF=0" (other distances the same way)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab.sh chirpz3000 "default go-dsp_amd/lib_pf0" 2 || exit $?
for L in default go-dsp_amd/lib_pf0; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  echo "== $L"; timeout -k 10 300 python scripts/bench_sizes.py 101 1021 2039 4093 4099 8191 8209 12289 > gpurun_out/sz.jsonl 2>&1 || exit $?
  grep '"chirpz": true' gpurun_out/sz.jsonl | python -c "import sys,json;[print(d['n'],d['ms']) for d in map(json.loads,sys.stdin)]"
done
