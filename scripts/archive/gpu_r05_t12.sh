# Round 5, late: more lengths' fused Pwelch on lists of their own (lib_t1 /
# lib_t2 via specspw: tools/spec_candidates.py's two best lists of as many or
# one more pass) against their FFT lists; half overlap, rocprofv3 kernel
# traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PW="4800:2400 5120:2560 3600:1800 1600:800 1800:900 1920:960 960:480 500:250 625:312 375:187 250:125 200:100 320:160 1152:576"
for r in 1 2; do
for L in default lib_t1 lib_t2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_t12_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/t12_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/t12_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_t12_$L.$r/run_kernel_trace.csv
done
done
