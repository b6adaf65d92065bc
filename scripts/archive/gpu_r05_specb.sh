# Round 5: radix lists with a higher per-pass thread occupancy for the
# compute-bound fused Pwelch (lib_specb: 2000 25 20 4, 2400 20 15 8, 1200 25
# 12 4, 800 25 8 4) against the compiled ones (25 5 16, 25 6 16, 25 3 16,
# 25 2 16): the batched FFT (HBM-bound), the fused Pwelch and Rader 1201.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_specb/libgdspfft.so timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "mixed or pwelch or Pwelch or rader or jit or sizes" > gpurun_out/r05/pytest_specb.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05/pytest_specb.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_specb; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py 800 1200 2000 2400 > $R/gpurun_out/r05/specb_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/specb_fft_$L.$r.jsonl; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_specb_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 800:400 1200:600 2000:1000 2400:1200 2000:0 > $R/gpurun_out/r05/specb_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/specb_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_specb_$L.$r/run_kernel_trace.csv
  timeout -k 10 300 python3 $R/scripts/bench_rader.py 1201 > $R/gpurun_out/r05/specb_rader_$L.$r.jsonl 2>&1; echo "== rader $L $r rc=$?"
done
done
cd $R && for f in gpurun_out/r05/specb_fft_*.jsonl gpurun_out/r05/specb_rader_*.jsonl; do echo "== $f"; cat $f; done
