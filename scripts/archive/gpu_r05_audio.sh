# Round 5, late: other lists as the fused Pwelch's own for the 44.1 kHz frame
# lengths 4410 / 2940 / 5880 / 2646 (lib_a1, lib_a2 via specspw) against their
# FFT lists; half overlap, rocprofv3 kernel traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_a1 lib_a2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_au_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 4410:2205 2940:1470 5880:2940 2646:1323 > $R/gpurun_out/r05/au_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/au_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_au_$L.$r/run_kernel_trace.csv
done
done
