# output-split chirp-z: parts of a row in adjacent blocks (default) against
# the part-major grid (lib_ymaj: scripts/build_variant.sh ymaj -DGDSP_BLU_PARTS_YMAJOR=1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "output_parts or chirpz or prime or fft2_vs_oracle" > gpurun_out/parts_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/parts_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for L in default go-dsp_amd/lib_ymaj; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
  timeout -k 10 300 python scripts/bench_sizes.py 8209 10007 11003 12289 13999 14563 > gpurun_out/sz.jsonl 2>&1 || exit $?
  echo "$L $(grep '"chirpz": false' gpurun_out/sz.jsonl | python -c "import sys,json;print(' '.join('%d:%.3f'%(d['n'],d['ms']) for d in map(json.loads,sys.stdin)))")"
done
done
