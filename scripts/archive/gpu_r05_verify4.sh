# Round 5, after the fused-Pwelch-only list (specspw) and the 2000 / 2400 /
# 1500 lists: the whole GPU suite (with test_pwelch_every_specialisation), the
# Pwelch NFFT cases under rocprofv3 kernel traces, and the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_verify4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify4.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
CASES="64:32 64:0 128:64 128:0 256:0 256:128 512:0 512:256 1024:0 1024:512 2048:0 2048:1024 4096:0 4096:1024 4096:2048 8192:4096 16384:8192 480:240 800:400 1000:500 1200:600 1500:700 1536:768 2000:1000 2205:1102 2400:1200 2880:1440 3000:1500 3840:1920 4500:2250 6000:3000 8000:4000"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pwfinal -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/r05/pwfinal.log 2>&1; rc=$?
echo "pw rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/pwfinal.log; exit $rc; }
python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pwfinal/run_kernel_trace.csv
cd $R && timeout -k 10 600 python3 bench.py > gpurun_out/r05/bench_final.json 2> gpurun_out/r05/bench_final.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r05/bench_final.json
