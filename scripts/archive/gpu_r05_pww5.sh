# Round 5: the Pwelch kernels as changed this session (wave kernel: unmasked
# full groups, no prefetch, three waves per SIMD for half overlap; NFFT 4096
# with any other overlap on the row kernel's structure; the fused mixed-radix
# kernel's unmasked loads) against the same sources before (lib_head) — GPU
# tests, then the Pwelch NFFT cases under rocprofv3 kernel traces, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch or rader or primes" > gpurun_out/r05/pytest_pww5.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pww5.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:0 2048:1024 4096:0 4096:1024 4096:2048 1000:500 3000:1500 2000:1000 1536:768 480:240 6000:3000"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_head; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pww5_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/r05/pww5_$L.$r.log 2>&1; rc=$?
  echo "== $L round $r rc=$rc"; [ $rc -eq 0 ] || { tail -20 $R/gpurun_out/r05/pww5_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pww5_$L.$r/run_kernel_trace.csv > $R/gpurun_out/r05/pww5_$L.$r.txt
done
done
cd $R && paste gpurun_out/r05/pww5_default.1.txt gpurun_out/r05/pww5_lib_head.1.txt | awk '{print $0}' | cut -c1-200
