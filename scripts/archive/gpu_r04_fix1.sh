set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out


bash scripts/gpu_r04_mix3000.sh
