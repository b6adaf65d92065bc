# Round 5, late: F = 8192 half-overlap Pwelch held to four waves per SIMD with the
# window from L1/L2 (pwelch_half_kernel<13, 1, 4, 4>: 128 VGPRs, 62 spilled, two
# workgroups per CU; lib_h13) against <13, 2, 1, 4> (186 VGPRs, window in LDS,
# one workgroup per CU); rocprofv3 kernel traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_h13; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_h13_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 8192:4096 > $R/gpurun_out/r05/h13_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/h13_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_h13_$L.$r/run_kernel_trace.csv
done
done
