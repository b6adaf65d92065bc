# Round 5, late: the 6000 fused Pwelch (15 5 5 16, seven-wave workgroups) held
# to four waves per SIMD so that two workgroups share a CU (lib_w4: 128 VGPRs,
# 32 spilled) against the compiler's 142 VGPRs (one workgroup per CU); two
# alternating rounds, rocprofv3 kernel traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_w4; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_w4_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 6000:3000 > $R/gpurun_out/r05/w4_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/w4_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_w4_$L.$r/run_kernel_trace.csv
done
done
