# Round 5, late: the short lengths' fused Pwelch on lists of their own
# (lib_c1 / lib_c2 via specspw: tools/spec_candidates.py's best untried lists
# of as many or one more pass) against their FFT lists; half overlap,
# rocprofv3 kernel traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PW="100:50 120:60 150:75 240:120 300:150 480:240 735:367 900:450 1000:500 1323:661 160:80 360:180 720:360 1125:562 1200:600 1470:735 1764:882"
for r in 1 2; do
for L in default lib_c1 lib_c2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_c12_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/c12_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/c12_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_c12_$L.$r/run_kernel_trace.csv
done
done
