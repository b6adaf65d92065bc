# Round 5: after the 4000 / 6000 Pwelch-only lists: the Pwelch and mixed-radix
# GPU tests, and the smooth-NFFT Pwelch cases under rocprofv3 kernel traces.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pwelch or Pwelch or mixed or specialisation" > gpurun_out/r05/pytest_verify5.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify5.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pwsm2 -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 3000:1500 4000:2000 6000:3000 > $R/gpurun_out/r05/pwsm2.log 2>&1; rc=$?
echo "pw rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/pwsm2.log; exit $rc; }
python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pwsm2/run_kernel_trace.csv
