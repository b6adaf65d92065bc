# Round 6: the VERDICT r05 named lengths (scripts/sweep_nonsmooth.py's default
# list) at the final sources, production and forced chirp-z plans.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06v
cd $R
python3 tools/source_stamp.py > gpurun_out/r06v/source_stamp.json
timeout -k 10 600 python3 scripts/sweep_nonsmooth.py > gpurun_out/r06v/nonsmooth_sweep.jsonl 2> gpurun_out/r06v/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06v/sweep.err; exit $rc; }
