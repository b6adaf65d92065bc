# Round 5: radix lists 1000 25 20 2 and 1500 25 15 4 (lib_specc) against 10 10 10 / 15 10 10:
# the fused Pwelch, the batched FFT and four-step lengths with rows of 1000.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_specc/libgdspfft.so timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "mixed or pwelch or Pwelch or rader or jit or sizes" > gpurun_out/r05/pytest_specc.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05/pytest_specc.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_specc; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py 1000 1500 30000 1000000 > $R/gpurun_out/r05/specc_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/specc_fft_$L.$r.jsonl; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_specc_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 1000:500 1500:750 1000:0 1500:0 > $R/gpurun_out/r05/specc_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/specc_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_specc_$L.$r/run_kernel_trace.csv
done
done
cd $R && for f in gpurun_out/r05/specc_fft_*.jsonl ; do echo "== $f"; cat $f; done
