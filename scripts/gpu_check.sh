set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; rc=$?
echo "prof rc=$rc"; find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
exit $rc
