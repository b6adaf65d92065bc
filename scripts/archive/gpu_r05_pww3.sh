# Round 5: wave Pwelch kernel with F = 2048 (two-wave workgroups) and the PF
# policy; the three-wave NFFT 4096 experiment (development build) under a
# kernel trace beside the product row kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch or shuffle or wave_kernel or three_wave" > gpurun_out/r05/pytest_pww3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pww3.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:0 2048:1024"
for r in 1 2; do
for L in default lib_pwoff; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/$L/libgdspfft.so
  echo "== $L round $r"
  timeout -k 10 300 python -u scripts/bench_pwelch.py $CASES > gpurun_out/r05/pww3_$L.$r.jsonl 2>gpurun_out/r05/pww3_$L.err; rc=$?
  cat gpurun_out/r05/pww3_$L.$r.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/r05/pww3_$L.err; exit $rc; }
done
done
unset GDSP_LIB
cd /tmp && export TMPDIR=/tmp
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r05/prof_pw4096dev -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_pw4096_dev.py > $GRAFT_REPO_ROOT/gpurun_out/r05/pw4096dev.log 2>&1; rc=$?
echo "prof rc=$rc"; cat $GRAFT_REPO_ROOT/gpurun_out/r05/pw4096dev.log | tail -5; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && python3 tools/trace_cases.py gpurun_out/r05/prof_pw4096dev/run_kernel_trace.csv
