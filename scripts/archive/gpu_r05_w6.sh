# Round 5, late: per-list register caps, second set (lib_w6: 160 at four waves per SIMD, 1000 at five, 150 882 4410 2880 2560 at three)
# against the compiler's counts; two alternating rounds, rocprofv3 traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_w6; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_w6_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 160:80 150:75 1000:500 882:441 4410:2205 2880:1440 2560:1280 > $R/gpurun_out/r05/w6_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/w6_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_w6_$L.$r/run_kernel_trace.csv
done
done
