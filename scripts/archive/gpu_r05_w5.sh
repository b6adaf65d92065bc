# Round 5, late: per-list register caps for the fused Pwelch (lib_w5: 4500
# 15 20 15 and 2000 10 10 20 at four waves per SIMD, 2400 15 16 10 at three)
# against the compiler's counts; two alternating rounds, rocprofv3 traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_w5; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_w5_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 4500:2250 2000:1000 2400:1200 3000:1500 > $R/gpurun_out/r05/w5_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/w5_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_w5_$L.$r/run_kernel_trace.csv
done
done
