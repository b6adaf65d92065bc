# Round 5: the fused mixed-radix Pwelch kernel — the next pair by LDS-DMA for
# radix-25 first passes, direct unconditional loads elsewhere (default),
# against the round's earlier kernel
# (lib_head); Pwelch GPU tests first. Kernel times from rocprofv3 traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pwf.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pwf.log; [ $rc -eq 0 ] || exit $rc
CASES="1000:500 3000:1500 2000:1000 1500:700 1536:768 480:240 2205:1102 6000:3000 810:400 1000:0"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_head; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pwf_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/r05/pwf_$L.$r.log 2>&1; rc=$?
  echo "== $L round $r rc=$rc"; [ $rc -eq 0 ] || { tail -20 $R/gpurun_out/r05/pwf_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pwf_$L.$r/run_kernel_trace.csv > $R/gpurun_out/r05/pwf_$L.$r.txt
done
done
cd $R && for L in default lib_head; do echo "== $L"; cat gpurun_out/r05/pwf_$L.2.txt; done
