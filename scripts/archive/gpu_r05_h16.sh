# Round 5, late: F = 16384 half-overlap Pwelch with 16 points per thread
# (pwelch_half_kernel<14, 1, 1, 4>: 1024 threads, 128 VGPRs, 67 spilled, four
# waves per SIMD; lib_h16) against 32 (<14, 1, 1, 5>: 512 threads, 256 VGPRs,
# 123 spilled, two waves), rocprofv3 kernel traces, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_h16; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_h16_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 16384:8192 8192:4096 > $R/gpurun_out/r05/h16_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/h16_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_h16_$L.$r/run_kernel_trace.csv
done
done
