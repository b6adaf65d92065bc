# Round 5, late: four-pass lists as the fused Pwelch's own (specspw) for 16
# more compiled lengths (lib_s1 / lib_s2: tools/spec_candidates.py's two best
# four-pass lists each) against their FFT lists; half overlap, rocprofv3
# kernel traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PW="400:200 441:220 750:375 768:384 1440:720 1875:937 2160:1080 2250:1125 2500:1250 2560:1280 3072:1536 3125:1562 3750:1875 5000:2500 6400:3200 7500:3750"
for r in 1 2; do
for L in default lib_s1 lib_s2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_s12_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/s12_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/s12_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_s12_$L.$r/run_kernel_trace.csv
done
done
