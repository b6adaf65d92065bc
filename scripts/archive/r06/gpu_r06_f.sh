# Round 6: SQ passes (VALU / LDS / wait shares) of the kind-8 and kind-7
# kernels at the bench shapes (pfa3027, prime3001).
set -o pipefail
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
python3 $GRAFT_REPO_ROOT/tools/source_stamp.py > $GRAFT_REPO_ROOT/gpurun_out/source_stamp.json
bash $GRAFT_REPO_ROOT/scripts/gpu_sq.sh pfa3027 prime3001
