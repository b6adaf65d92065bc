# Round 6: the kind-8 kernel with rows per workgroup held to 40 KiB of LDS,
# against the round's first calibration (profiles/r06/pfa_calib.jsonl):
# the same 150 lengths without the race, then the SQ passes of pfa3027.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06e
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 900 python -u scripts/sweep_pfa_calib.py --no-race > gpurun_out/r06e/pfa_calib_tpw40.jsonl 2> gpurun_out/r06e/calib.err; rc=$?
echo "calib rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06e/calib.err; exit $rc; }
