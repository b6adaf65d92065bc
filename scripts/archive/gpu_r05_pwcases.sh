# Round 5: Pwelch GPU tests (also on lib_pwlay1: the wave kernels' exchanges
# in the linear padded layout), then every Pwelch NFFT case of
# scripts/bench_pwelch.py under rocprofv3 kernel traces, default and
# lib_pwlay1 alternating, two rounds (tools/pwelch_cases.py).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pwcases.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_pwcases.log; [ $rc -eq 0 ] || exit $rc
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_pwlay1/libgdspfft.so timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pwelch or Pwelch" > gpurun_out/r05/pytest_pwlay1.log 2>&1; rc=$?
echo "pytest lay1 rc=$rc"; tail -3 gpurun_out/r05/pytest_pwlay1.log; [ $rc -eq 0 ] || exit $rc
CASES="64:32 128:64 256:0 256:128 512:256 1024:0 1024:512 2048:0 2048:1024 4096:0 4096:1024 4096:2048 8192:4096 16384:8192 480:240 1000:500 1500:700 1536:768 2000:1000 2205:1102 3000:1500 6000:3000"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_pwlay1; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  D=prof_pwcases.$r; [ $L = default ] || D=prof_pwlay1.$r
  timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/$D -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/r05/$D.log 2>&1; rc=$?
  echo "== $L round $r rc=$rc"; [ $rc -eq 0 ] || { tail -20 $R/gpurun_out/r05/$D.log; exit $rc; }
done
done
