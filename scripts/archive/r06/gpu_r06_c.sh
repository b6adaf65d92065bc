# Round 6: kind-8 calibration sweep (prime-factor Rader against chirp-z).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06c
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1000 python -u scripts/sweep_pfa_calib.py > gpurun_out/r06c/pfa_calib.jsonl 2> gpurun_out/r06c/calib.err; rc=$?
echo "calib rc=$rc"; tail -3 gpurun_out/r06c/calib.err; exit $rc
