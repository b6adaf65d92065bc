# Pwelch cases of scripts/bench_pwelch.py with per-dispatch kernel times
# (rocprofv3 kernel trace), summarised per case by tools/trace_cases.py.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_pw -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_pwelch.py > $GRAFT_REPO_ROOT/gpurun_out/prof_pw.log 2>&1; rc=$?
echo "prof rc=$rc"; cat $GRAFT_REPO_ROOT/gpurun_out/prof_pw.log | tail -12; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && python3 tools/trace_cases.py gpurun_out/prof_pw/run_kernel_trace.csv
