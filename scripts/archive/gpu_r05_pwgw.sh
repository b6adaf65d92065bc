# Round 5: NFFT 2048 half overlap with the window read from L1/L2 instead of
# LDS (21 KiB per workgroup) and three waves per SIMD (lib_pwgw) against the
# kept kernel; Pwelch tests on the variant first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_pwgw/libgdspfft.so timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pwgw.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r05/pytest_pwgw.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2 3; do
for L in default lib_pwgw; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pwgw_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 2048:1024 2048:0 2048:512 > $R/gpurun_out/r05/pwgw_$L.$r.log 2>&1; rc=$?
  echo "== $L round $r rc=$rc"; [ $rc -eq 0 ] || { tail -20 $R/gpurun_out/r05/pwgw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pwgw_$L.$r/run_kernel_trace.csv
done
done
