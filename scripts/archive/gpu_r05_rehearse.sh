# Round 5: the driver's N > 1 form rehearsed on a one-GPU box — the plain
# `bench.py --gpus 2` (it spawns its two ranks) over gloo, both ranks on
# cuda:0, every nested config included (prime3001 and pwelch_default new).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
GDSP_DIST_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/r05/rehearse_gloo2_default.json 2> gpurun_out/r05/rehearse_gloo2_default.err; rc=$?
echo "rc=$rc"; head -c 600 gpurun_out/r05/rehearse_gloo2_default.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/r05/rehearse_gloo2_default.err; exit $rc; }
