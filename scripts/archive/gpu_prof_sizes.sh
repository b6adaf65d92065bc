# Parity tests selected by $K, then a rocprofv3 kernel-stats profile of
# scripts/bench_sizes.py for the lengths given as arguments.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "${K:-fourstep or plan_kinds}" > gpurun_out/ps_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/ps_pytest.log)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sizes -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_sizes.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_sizes.log 2>&1; rc=$?
echo "prof rc=$rc"; cat $GRAFT_REPO_ROOT/gpurun_out/prof_sizes.log | grep '^{'
exit $rc
