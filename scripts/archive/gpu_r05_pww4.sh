# Round 5: the wave Pwelch kernel with unmasked full groups (buffer loads from
# a per-group scalar descriptor) against the previous kernel (lib_pwold) and
# two no-prefetch three-waves-per-SIMD variants (lib_pwb: 3072 waves, lib_pwc:
# 2048), per-case kernel times from rocprofv3 kernel traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pww4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pww4.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:0 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:0 2048:1024 200:100 300:0"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_pwold lib_pwb lib_pwc; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pww4_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/r05/pww4_$L.$r.log 2>&1; rc=$?
  echo "== $L round $r rc=$rc"; [ $rc -eq 0 ] || { tail -20 $R/gpurun_out/r05/pww4_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pww4_$L.$r/run_kernel_trace.csv | tee $R/gpurun_out/r05/pww4_$L.$r.txt
done
done
