# Round 6, first session: the GPU suite at the round's first changes
# (negative-Noverlap guards, full-size Pwelch vs the oracle, shim without a
# host path), then the non-smooth length sweep before any new kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06a
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 300 python -u scripts/sweep_nonsmooth.py > gpurun_out/r06a/nonsmooth_sweep_start.jsonl 2> gpurun_out/r06a/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r06a/sweep.err; exit $rc; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "fullsize or negative_noverlap or shim_replay or pwelch_random" > gpurun_out/r06a/pytest_sel.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r06a/pytest_sel.log; exit $rc
